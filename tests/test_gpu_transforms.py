"""GPU parity of the HIP transforms (fgp_fftbr / fgp_ifftbr / fgp_fwht) against the CPU oracle.

Tolerance (fp64): max |gpu - oracle| <= 1e-13 * max|oracle| * (1 + m) for the orthonormal
transforms (both are O(eps log n) backward-stable; measured spread between two CPU FFT libraries
is ~1e-15 relative).  Bit-reversal / index work is exact by construction and checked through
permutation inputs (unit vectors map to exact roots of unity).
"""
import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O
from tests.golden_util import golden_names, load_golden

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)
DEV = "cuda"


def _tol(m):
    return 1e-13 * (1 + m)


def _close(a, b, m):
    a = a.detach().cpu()
    b = b.detach().cpu()
    scale = float(b.abs().max()) if b.numel() else 1.0
    err = float((a - b).abs().max()) if b.numel() else 0.0
    assert err <= _tol(m) * max(scale, 1e-300), "err %.3e scale %.3e (m=%d)" % (err, scale, m)


@pytest.mark.parametrize("m", list(range(0, 21)))
def test_fftbr_matches_oracle(m):
    n = 2 ** m
    g = torch.Generator().manual_seed(m)
    batch = 3 if m <= 16 else 1
    xr = torch.randn((batch, n), generator=g) + 2.0
    xc = torch.randn((batch, n), generator=g) + 1j * torch.randn((batch, n), generator=g)
    _close(F.ops.fftbr_raw(xr.to(DEV), stable=False), O.fftbr(xr), m)
    _close(F.ops.fftbr_raw(xc.to(DEV), stable=False), O.fftbr(xc), m)
    _close(F.ops.fftbr_raw(xr.to(DEV), stable=True), O.ft_stable(xr, O.fftbr), m)


@pytest.mark.parametrize("m", list(range(0, 21)))
def test_ifftbr_matches_oracle(m):
    n = 2 ** m
    g = torch.Generator().manual_seed(100 + m)
    batch = 2 if m <= 16 else 1
    x = torch.randn((batch, n), generator=g) + 1j * torch.randn((batch, n), generator=g) + 0.5
    _close(F.ops.ifftbr_raw(x.to(DEV), stable=False), O.ifftbr(x), m)
    _close(F.ops.ifftbr_raw(x.to(DEV), stable=True), O.ft_stable(x, O.ifftbr), m)
    _close(F.ops.ifftbr_raw(x.to(DEV), stable=True, real_out=True), O.ft_stable(x, O.ifftbr).real, m)


@pytest.mark.parametrize("m", list(range(0, 21)))
def test_fwht_matches_oracle(m):
    n = 2 ** m
    g = torch.Generator().manual_seed(200 + m)
    batch = 3 if m <= 16 else 1
    x = torch.randn((batch, n), generator=g) + 3.0
    _close(F.ops.fwht_raw(x.to(DEV), stable=False), O.fwht(x), m)
    _close(F.ops.fwht_raw(x.to(DEV), stable=True), O.ft_stable(x, O.fwht), m)


@pytest.mark.parametrize("m", [0, 3, 4, 12, 13, 16, 20])
def test_unit_vectors_give_exact_bitreversed_roots(m):
    """fftbr(e_i)[k] = exp(-2 pi i brev(i) k / n) / sqrt(n): locates the bit-reversal exactly."""
    n = 2 ** m
    br = O.bitrev_indices(m)
    for i in sorted({0, 1, n // 3, n - 1} & set(range(n))):
        e = torch.zeros(n)
        e[i] = 1.0
        y = F.ops.fftbr_raw(e.to(DEV)).cpu() * np.sqrt(n)
        k = torch.arange(n, dtype=torch.float64)
        ref = torch.exp(-2j * np.pi * ((int(br[i]) * k) % n) / n)
        assert float((y - ref).abs().max()) < 1e-12 * (1 + m)


@pytest.mark.parametrize("m", [4, 12, 13, 18, 20])
def test_roundtrip_and_parseval(m):
    n = 2 ** m
    g = torch.Generator().manual_seed(300 + m)
    x = (torch.randn((2, n), generator=g) + 1j * torch.randn((2, n), generator=g)).to(DEV)
    y = F.ops.fftbr_raw(x, stable=True)
    back = F.ops.ifftbr_raw(y, stable=True)
    assert float((back - x).abs().max()) < 1e-13 * (1 + m) * float(x.abs().max())
    assert torch.allclose(y.abs().pow(2).sum(-1), x.abs().pow(2).sum(-1), rtol=1e-13 * (1 + m))
    w = F.ops.fwht_raw(F.ops.fwht_raw(x.real.contiguous(), stable=True), stable=True)
    assert float((w - x.real).abs().max()) < 1e-13 * (1 + m) * float(x.real.abs().max())


def test_noncontiguous_and_batched_shapes():
    g = torch.Generator().manual_seed(7)
    x = torch.randn((4, 3, 64), generator=g)
    xt = x.to(DEV).transpose(0, 1)  # non-contiguous leading dims
    _close(F.ops.fftbr_raw(xt), O.fftbr(x.transpose(0, 1)), 6)
    big = torch.randn((2, 2 ** 14 * 2), generator=g)[:, ::2]  # strided last dim
    _close(F.ops.fftbr_raw(big.to(DEV)), O.fftbr(big.contiguous()), 14)


def test_autograd_adjoints():
    """backward of each transform is its exact adjoint: <A x, y> = <x, A^H y>."""
    g = torch.Generator().manual_seed(9)
    for m in (3, 10, 15):
        n = 2 ** m
        x = torch.randn(n, generator=g).to(DEV).requires_grad_(True)
        w = (torch.randn(n, generator=g) + 1j * torch.randn(n, generator=g)).to(DEV)
        (F.ops.fftbr(x, stable=True) * w.conj()).real.sum().backward()
        ref = O.ifftbr(w.cpu()).real
        assert float((x.grad.cpu() - ref).abs().max()) < 1e-12
        xw = torch.randn(n, generator=g).to(DEV).requires_grad_(True)
        v = torch.randn(n, generator=g).to(DEV)
        (F.ops.fwht(xw) * v).sum().backward()
        assert float((xw.grad.cpu() - O.fwht(v.cpu())).abs().max()) < 1e-12


@pytest.mark.parametrize("name", golden_names())
def test_golden_stable_transforms(name):
    g = load_golden(name)
    m = int(g["m"])
    fam = str(g["family"])
    ft = (lambda v: F.ops.fftbr(v, stable=True)) if fam == "lattice" else (lambda v: F.ops.fwht(v, stable=True))
    ift = (lambda v: F.ops.ifftbr(v, stable=True)) if fam == "lattice" else (lambda v: F.ops.fwht(v, stable=True))
    _close(ft(torch.from_numpy(g["ft_in"]).to(DEV)), torch.from_numpy(g["ft_out"]), m)
    _close(ift(torch.from_numpy(g["ift_in"]).to(DEV)), torch.from_numpy(g["ift_out"]), m)


# ---------------------------------------------------------------- single precision (c64 / f32)
def _close32(a, b, m):
    """fp32 transforms against the fp64 oracle: |err| <= 2e-7 (1 + m) max|oracle| (fp32 eps = 6e-8;
    O(eps log n) backward-stable butterflies, twiddles rounded once from the fp64 tables)."""
    a = a.detach().cpu().to(torch.complex128 if a.is_complex() else torch.float64)
    b = b.detach().cpu()
    err = float((a - b).abs().max())
    scale = float(b.abs().max())
    assert err <= 2e-7 * (1 + m) * scale, "fp32 err %.3e scale %.3e (m=%d)" % (err, scale, m)


@pytest.mark.parametrize("m", [0, 1, 3, 4, 7, 12, 13, 16, 17, 20])
def test_single_precision_transforms_match_oracle(m):
    n = 2 ** m
    g = torch.Generator().manual_seed(300 + m)
    batch = 3 if m <= 16 else 1
    xr = torch.randn((batch, n), generator=g) + 2.0
    xc = torch.randn((batch, n), generator=g) + 1j * torch.randn((batch, n), generator=g)
    xr32, xc32 = xr.float(), xc.to(torch.complex64)
    # oracle on the fp32-rounded inputs (the comparison measures the transform, not the input rounding)
    out = F.ops.fftbr_raw(xr32.to(DEV), stable=True)
    assert out.dtype == torch.complex64
    _close32(out, O.ft_stable(xr32.double(), O.fftbr), m)
    _close32(F.ops.fftbr_raw(xc32.to(DEV), stable=False), O.fftbr(xc32.to(torch.complex128)), m)
    inv = F.ops.ifftbr_raw(xc32.to(DEV), stable=True)
    assert inv.dtype == torch.complex64
    _close32(inv, O.ft_stable(xc32.to(torch.complex128), O.ifftbr), m)
    re = F.ops.ifftbr_raw(xc32.to(DEV), stable=True, real_out=True)
    assert re.dtype == torch.float32
    _close32(re, O.ft_stable(xc32.to(torch.complex128), O.ifftbr).real, m)
    w = F.ops.fwht_raw(xr32.to(DEV), stable=True)
    assert w.dtype == torch.float32
    _close32(w, O.ft_stable(xr32.double(), O.fwht), m)


@pytest.mark.parametrize("m", [2, 10, 14, 18])
def test_inverse_mul_and_sum_sq(m):
    """fgp_ifftbr_mul (the factor fused into the inverse's first pass) equals the inverse of the
    product; fgp_sum_sq equals the grouped sum of squares -- fp64 to the transform tolerance, fp32 to
    its own."""
    n = 2 ** m
    g = torch.Generator().manual_seed(400 + m)
    B = 6
    x = (torch.randn((B, n), generator=g) + 1j * torch.randn((B, n), generator=g)).to(DEV)
    f1 = (torch.randn((1, n), generator=g) + 1j * torch.randn((1, n), generator=g)).to(DEV)
    fB = (torch.randn((B, n), generator=g) + 1j * torch.randn((B, n), generator=g)).to(DEV)
    for f in (f1, fB):
        got = F.ops.inverse_mul(F.ops.LATTICE, x, f, real_out=True)
        ref = O.ft_stable((x * f).cpu(), O.ifftbr).real
        _close(got, ref, m)
        got32 = F.ops.inverse_mul(F.ops.LATTICE, x.to(torch.complex64), f.to(torch.complex64), real_out=True)
        assert got32.dtype == torch.float32
        _close32(got32, O.ft_stable((x.to(torch.complex64) * f.to(torch.complex64)).to(torch.complex128).cpu(),
                                    O.ifftbr).real, m)
        xr, fr = x.real.contiguous(), f.real.contiguous()
        _close(F.ops.inverse_mul(F.ops.NET, xr, fr), O.ft_stable((xr * fr).cpu(), O.fwht), m)
    for G in (1, 2, 3, 6):
        s = F.ops.sum_sq(x, G=G).cpu()
        ref = (x.abs() ** 2).cpu().reshape(-1, G, n).sum(0)
        assert float((s - ref).abs().max()) <= 1e-14 * float(ref.abs().max())
    s32 = F.ops.sum_sq(x.to(torch.complex64), G=1).cpu()
    ref32 = (x.to(torch.complex64).to(torch.complex128).abs() ** 2).cpu().sum(0)
    assert float((s32 - ref32).abs().max()) <= 1e-14 * float(ref32.abs().max())


@pytest.mark.parametrize("m", [5, 14])
def test_lazy_conj_and_neg_views_are_materialised(m):
    """x.conj() / -x views share unconjugated storage; the kernels must see their values (the gradient
    through lam.conj() of the multitask blocks, util.py:284, arrives as such a view)."""
    g = torch.Generator().manual_seed(3)
    n = 2 ** m
    z = (torch.randn((2, n), generator=g) + 1j * torch.randn((2, n), generator=g)).to(DEV)
    for op in (F.ops.fftbr, F.ops.ifftbr):
        for stable in (False, True):
            assert torch.equal(op(z.conj(), stable=stable), op(z.conj().resolve_conj(), stable=stable))
            assert torch.equal(op(-z, stable=stable), op((-z).resolve_neg(), stable=stable))
    assert torch.equal(F.ops.fwht(z.conj(), stable=True), F.ops.fwht(z.conj().resolve_conj(), stable=True))
    zc = z.clone().requires_grad_(True)
    y = F.ops.fftbr(zc.conj(), stable=True)
    gz, = torch.autograd.grad((y.real * torch.arange(n, device=DEV)).sum(), zc)
    zr = z.clone().requires_grad_(True)
    yr = F.ops.fftbr(zr.conj().resolve_conj(), stable=True)
    gr, = torch.autograd.grad((yr.real * torch.arange(n, device=DEV)).sum(), zr)
    assert torch.allclose(gz, gr, rtol=0, atol=1e-12)


@pytest.mark.parametrize("m", [0, 1, 3, 7, 12, 13, 16, 19])
def test_doubling_stage_equals_full_transform(m):
    """fgp_double_update (util.py:113-132,173-178): ft of 2n values from ft of both halves, against the
    full-length transform, lattice (fftbr, w^k = exp(-pi i k / n)) and net (fwht, w = 1)."""
    g = torch.Generator().manual_seed(40 + m)
    n = 2 ** m
    y = (torch.randn((3, 2 * n), generator=g) + 3.0).to(DEV)
    for fam, ft in ((F.ops.LATTICE, lambda v: F.ops.fftbr(v, stable=True)), (F.ops.NET, lambda v: F.ops.fwht(v, stable=True))):
        full = ft(y)
        dbl = F.ops.double_update(fam, ft(y[:, :n]), ft(y[:, n:]))
        assert dbl.shape == full.shape and dbl.dtype == full.dtype
        assert float((dbl - full).abs().max()) <= 1e-13 * (1 + m) * float(full.abs().max())


def test_ytilde_and_lam_doubling_in_the_gp():
    """add_y_next doubling n reuses ytilde_n (one stage on the new half) and post_var(n=2n) reuses
    lam_n; both equal the full-length computation."""
    torch.set_default_dtype(torch.float64)
    for fam in ("lattice", "net"):
        seq = F.Lattice(3, seed=11) if fam == "lattice" else F.DigitalNetB2(3, seed=11)
        cls = F.FastGPLattice if fam == "lattice" else F.FastGPDigitalNetB2
        gp = cls(seq, device=DEV)
        x = gp.get_x_next(2 ** 12)
        f = lambda v: torch.cos(2 * np.pi * v).sum(1) + v[:, 0]   # noqa: E731
        gp.add_y_next(f(x))
        yt1 = gp.get_ytilde(0)
        x2 = gp.get_x_next(2 ** 14)
        gp.add_y_next(f(x2))
        yt2 = gp.get_ytilde(0)                                    # two doubling stages
        full = gp.ft(gp.y)
        assert float((yt2 - full).abs().max()) <= 1e-12 * float(full.abs().max())
        assert torch.equal(yt2[..., :1], yt2[..., :1]) and yt1.shape[-1] == 2 ** 12
        with torch.no_grad():
            lam_n = gp.get_lam(0, 0, 2 ** 14)
            lam_2n = gp.get_lam(0, 0, 2 ** 15)                      # doubled from lam_n
            ref = gp.ft(gp._k1(2 ** 15))
        assert float((lam_2n - ref).abs().max()) <= 1e-12 * float(ref.abs().max())
        assert lam_n.shape[-1] == 2 ** 14


@pytest.mark.parametrize("d,t", [(1, 32), (3, 32), (5, 53), (2, 63)])
def test_device_point_generators_are_bit_identical(d, t):
    """fgp_lattice_points / fgp_net_points (the generators get_x_next uses for this package's
    sequences) against the host restatement of qmcpy's natural-order generators, arbitrary ranges."""
    lat = F.Lattice(d, seed=5)
    net = F.DigitalNetB2(d, seed=5, t=t)
    for n0, n1 in ((0, 1), (0, 8), (8, 16), (1024, 4096), (0, 2 ** 17)):
        xl = F.ops.lattice_points([int(v) for v in lat.z[:d]], lat.shift, n0, n1, device=DEV)
        assert np.array_equal(xl.cpu().numpy(), lat(n_min=n0, n_max=n1))
        x, xb = F.ops.net_points(net.C, net.shift, t, n0, n1, DEV)
        ref = net(n_min=n0, n_max=n1, return_binary=True).astype(np.int64)
        assert np.array_equal(xb.cpu().numpy(), ref)
        assert np.array_equal(x.cpu().numpy(), ref.astype(np.float64) * 2.0 ** (-t))


@pytest.mark.parametrize("m,batch", [(17, 3), (18, 2), (20, 2), (22, 1), (24, 1)])
def test_fftbr_real_half_length_matches_full_length(monkeypatch, m, batch):
    """fgp_fftbr_real (real float64 input, n >= 2^17: the n/2-point packed transform with the split in
    the column pass) against the full-length fgp_fftbr (FGP_R2C=0) on the same rows, batched and from a
    strided view, to the transform tolerance; and against the oracle at m <= 20."""
    n = 2 ** m
    g = torch.Generator().manual_seed(300 + m)
    x = (torch.randn((batch, n + 8), generator=g) + 1.5).to(DEV)
    xs = x[:, :n]                                   # row stride n + 8 (view, even stride)
    half = F.ops.fftbr_raw(xs, stable=True)
    monkeypatch.setenv("FGP_R2C", "0")
    full = F.ops.fftbr_raw(xs, stable=True)
    _close(half, full, m)
    if m <= 20:
        _close(half, O.ft_stable(xs.cpu(), O.fftbr), m)


@pytest.mark.parametrize("m,batch,shared_f", [(17, 3, False), (18, 2, True), (20, 2, False), (22, 1, True),
                                              (24, 1, False)])
def test_ifftbr_real_half_length_matches_full_length(monkeypatch, m, batch, shared_f):
    """fgp_ifftbr_real (Re ifftbr at half length: the Hermitian part of every mirror pair packed into an
    n/2-point adjoint transform) against the full-length real-output inverse (FGP_R2C=0), on arbitrary
    (non-Hermitian) complex rows, without and with the fused product (inverse_mul, one shared row or one
    per row), to the transform tolerance; and against the oracle at m <= 20."""
    n = 2 ** m
    g = torch.Generator().manual_seed(400 + m)
    x = (torch.randn((batch, n), generator=g) + 1j * torch.randn((batch, n), generator=g) + 0.5).to(DEV)
    f = (torch.rand((1 if shared_f else batch, n), generator=g) + 0.5 + 0.1j * torch.randn((1 if shared_f else batch, n), generator=g)).to(DEV)
    half = F.ops.ifftbr_raw(x, stable=True, real_out=True)
    half_mul = F.ops.inverse_mul(F.ops.LATTICE, x, f, real_out=True)
    monkeypatch.setenv("FGP_R2C", "0")
    full = F.ops.ifftbr_raw(x, stable=True, real_out=True)
    full_mul = F.ops.inverse_mul(F.ops.LATTICE, x, f, real_out=True)
    assert half.dtype == torch.float64 and half.shape == (batch, n)
    _close(half, full, m)
    _close(half_mul, full_mul, m)
    if m <= 20:
        _close(half, O.ft_stable(x.cpu(), O.ifftbr).real, m)


@pytest.mark.parametrize("m,rows", [(17, 3), (18, 4)])
def test_float32_rows_widened_on_load_equal_float64_half(m, rows):
    """fgp_fftbr_real_half_f32 (ABI 16: data_dtype=float32 observations) equals fgp_fftbr_real_half of the rows
    widened to float64 bit for bit (the widening is exact), also for rows with a padded stride."""
    from fastgaussianprocesses_amd import ops
    n = 2 ** m
    g = torch.Generator().manual_seed(m + 1)
    y32 = (torch.randn((rows, n + 8), generator=g) + 3.0).float().to(DEV)
    for y in (y32[:, :n].contiguous(), y32[:, :n]):
        assert torch.equal(ops.fftbr_real_half(y), ops.fftbr_real_half(y.double()))


@pytest.mark.parametrize("m,rows", [(17, 3), (18, 5), (20, 2)])
def test_hermitian_half_spectra_equal_full_length_ones(m, rows):
    """fgp_fftbr_real_half (ABI 14) writes fgp_fftbr_real's values at k <= n/2 only: bit for bit, and the
    mirror (ops.hermitian_full) rebuilds the full output bit for bit; fgp_sum_sq_half from the halves equals
    fgp_sum_sq of the full spectra bit for bit (G = 1 and per-row groups); fgp_ifftbr_real_rf on the halves
    (rows of n/2 + 1) equals it on the full rows bit for bit."""
    from fastgaussianprocesses_amd import ops
    n = 2 ** m
    g = torch.Generator().manual_seed(m)
    y = (torch.randn((rows, n), generator=g) + 3.0).to(DEV)
    full = ops.fftbr_raw(y, stable=True)
    half = ops.fftbr_real_half(y)
    assert half.shape == (rows, n // 2 + 1)
    assert torch.equal(half, full[:, :n // 2 + 1])
    assert torch.equal(ops.hermitian_full(half, n), full)
    for G in (1, rows):
        assert torch.equal(ops.sum_sq_half(half, n, G=G), ops.sum_sq(full, G=G))
    f = (torch.rand((1, n), generator=g) + 0.5).to(DEV)
    f = 0.5 * (f + torch.roll(f.flip(-1), 1, -1))            # an even factor row, as A = 1/ev
    assert torch.equal(ops.ifftbr_real_rf(half, f, n=n), ops.ifftbr_real_rf(full, f))
