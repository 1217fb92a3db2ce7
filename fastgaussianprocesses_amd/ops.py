"""Torch-facing operators over the C-ABI library (include/fgp_hip.h).

Every operator runs on the input tensors' HIP device, on torch's current stream, and raises if a
tensor is not on a HIP device: there is no CPU fallback.

Drop-in transforms (the plugin point `ft`/`ift` of AbstractFastGP, fastgps/abstract_fast_gp.py:26-27,
197-228, filled by qmcpy.fftbr_torch / ifftbr_torch / fwht_torch at fast_gp_lattice.py:224-225 and
fast_gp_digital_net_b2.py:226):
    fftbr(x)   = fft(x[..., bitrev], norm="ortho")          (complex128 out)
    ifftbr(x)  = ifft(x, norm="ortho")[..., bitrev]
    fwht(x)    = orthonormal Sylvester-order Walsh-Hadamard
all differentiable (backward = the exact adjoint transform, real part for real inputs).
With stable=True the mean-centring of AbstractFastGP.ft/ift happens inside the kernels.
"""
import functools
import math
import os

import numpy as np

import torch

from . import _native as N

LATTICE = 0
NET = 1


def require_device(t, what):
    if not t.is_cuda:
        raise RuntimeError("%s: tensor on %s; fastgaussianprocesses_amd runs only on a HIP device (MI355X) "
                           "and has no CPU fallback" % (what, t.device))


def log2_exact(n):
    n = int(n)
    if n < 1 or (n & (n - 1)) != 0:
        raise AssertionError("n = %d must be a power of 2" % n)
    return n.bit_length() - 1


def resolved(x):
    """x with torch's lazy conjugate / negation bits materialised: the kernels read raw memory, and a
    `.conj()` view (e.g. the gradient autograd hands through a conj) shares its unconjugated storage."""
    return x.resolve_conj().resolve_neg() if x.is_complex() else x.resolve_neg()


def _as_rows(x):
    """View x[..., n] as [batch, n] with unit inner stride; returns (rows, batch_stride)."""
    x = resolved(x)
    n = x.shape[-1]
    r = x.reshape(-1, n)
    if r.stride(-1) != 1 or (r.size(0) > 1 and r.stride(0) < n):
        r = r.contiguous()
    return r, (r.stride(0) if r.size(0) > 1 else n)


def _stream(t):
    return N.stream_ptr(t.device)


# ------------------------------------------------------------------------------------- transforms
def _single(x):
    """float32 / complex64 input selects the single-precision kernels (fgp_*_c64 / fgp_fwht_f32)."""
    return x.dtype in (torch.float32, torch.complex64)


def fftbr_raw(x, stable=True):
    """fftbr (+ AbstractFastGP.ft's centring when stable) along the last dim: complex128 out for
    float64 / complex128 input (fgp_fftbr), complex64 out for float32 / complex64 input (fgp_fftbr_c64)."""
    require_device(x, "fftbr")
    sp = _single(x)
    rdt, cdt = (torch.float32, torch.complex64) if sp else (torch.float64, torch.complex128)
    x = x.to(cdt) if x.is_complex() else x.to(rdt)
    shape = x.shape
    n = shape[-1]
    m = log2_exact(n)
    rows, bs = _as_rows(x)
    out = torch.empty(rows.shape, dtype=cdt, device=x.device)
    if stable and _real_half_length(x, m) and rows.data_ptr() % 16 == 0 and bs % 2 == 0:
        # real float64 input, 2^17 <= n <= 2^24: the half-length transform (fgp_fftbr_real, 40n instead
        # of 56n bytes per row; it centres every row / column internally, so only for stable=True --
        # stable=False keeps qmcpy.fftbr_torch's plain transform)
        work = torch.empty(rows.shape, dtype=cdt, device=x.device)
        N.call("fgp_fftbr_real", N.ptr(rows), bs, N.ptr(out), N.ptr(work), rows.size(0), m, _stream(x))
        return out.reshape(shape)
    N.call("fgp_fftbr_c64" if sp else "fgp_fftbr", N.ptr(rows), bs, 0 if x.is_complex() else 1, N.ptr(out),
           rows.size(0), m, int(stable), _stream(x))
    return out.reshape(shape)


def half_spectrum_ok(x):
    """fgp_fftbr_real_half applies to x: real float64 (or float32: widened on load) rows, 2^17 <= n <= 2^24
    (FGP_YT_HALF=0 / FGP_R2C=0 off)."""
    n = x.shape[-1]
    return (x.dtype in (torch.float64, torch.float32) and n >= 2 and (n & (n - 1)) == 0
            and 17 <= n.bit_length() - 1 <= 24 and rows_ok_env() and os.environ.get("FGP_YT_HALF", "1")[:1] != "0")


def fftbr_real_half(x):
    """The Hermitian half (k = 0 .. n/2) of the stable fftbr of real float64 rows x [*, n] -> complex128
    [*, n/2 + 1] (fgp_fftbr_real_half: fgp_fftbr_real's values there, half the bytes written)."""
    require_device(x, "fftbr_real_half")
    shape = x.shape
    n = shape[-1]
    m = log2_exact(n)
    f32 = x.dtype == torch.float32
    assert (x.dtype == torch.float64 or f32) and 17 <= m <= 24, "fftbr_real_half: float64 / float32 rows, 2^17 <= n <= 2^24"
    rows, bs = _as_rows(x)
    if rows.data_ptr() % 16 or bs % (4 if f32 else 2):
        rows, bs = rows.contiguous(), n
    H = n // 2 + 1
    out = torch.empty((rows.size(0), H), dtype=torch.complex128, device=x.device)
    work = torch.empty((rows.size(0), n), dtype=torch.complex128, device=x.device)
    N.call("fgp_fftbr_real_half_f32" if f32 else "fgp_fftbr_real_half", N.ptr(rows), bs, N.ptr(out), H, N.ptr(work),
           rows.size(0), m, _stream(x))
    return out.reshape(shape[:-1] + (H,))


def hermitian_full(xh, n):
    """[*, n/2 + 1] Hermitian half -> the full [*, n] spectrum (X_{n-k} = conj X_k)."""
    H = n // 2 + 1
    assert xh.shape[-1] == H
    full = torch.empty(xh.shape[:-1] + (n,), dtype=xh.dtype, device=xh.device)
    full[..., :H] = xh
    full[..., H:] = xh[..., 1:n // 2].flip(-1).conj()
    return full


def sum_sq_half(xh, n, G=1):
    """Y[g, k] = sum_r |X[r G + g, k]|^2 [G, n] from Hermitian halves xh [R G, n/2 + 1] complex128
    (fgp_sum_sq_half: sum_sq of the full spectra, bit for bit)."""
    require_device(xh, "sum_sq_half")
    rows, bs = _as_rows(xh)
    assert rows.dtype == torch.complex128 and rows.size(0) % G == 0
    out = torch.empty((G, n), dtype=torch.float64, device=xh.device)
    N.call("fgp_sum_sq_half", N.ptr(rows), bs, rows.size(0) // G, G, n, N.ptr(out), _stream(xh))
    return out


def _real_half_length(x, m):
    """fgp_fftbr_real applies: float64 real input, 17 <= m <= 24 (FGP_R2C=0 keeps the full-length path)."""
    return (x.dtype == torch.float64 and 17 <= m <= 24 and rows_ok_env())


def rows_ok_env():
    return os.environ.get("FGP_R2C", "2")[:1] != "0"


def ifftbr_raw(x, stable=True, real_out=False):
    """ifftbr along the last dim (fgp_ifftbr / fgp_ifftbr_c64 for complex64 input); real_out keeps
    only the real part (gram_matrix_solve's .real, util.py:343)."""
    require_device(x, "ifftbr")
    sp = _single(x)
    rdt, cdt = (torch.float32, torch.complex64) if sp else (torch.float64, torch.complex128)
    x = x.to(cdt)
    shape = x.shape
    n = shape[-1]
    m = log2_exact(n)
    rows, bs = _as_rows(x)
    if real_out and stable and not sp and 17 <= m <= 24 and rows_ok_env():
        # real part at half length (fgp_ifftbr_real): the Hermitian part through an n/2-point transform
        out = torch.empty(rows.shape, dtype=rdt, device=x.device)
        work = torch.empty(rows.shape, dtype=cdt, device=x.device)
        N.call("fgp_ifftbr_real", N.ptr(rows), bs, None, 0, N.ptr(out), n, N.ptr(work), rows.size(0), m, _stream(x))
        return out.reshape(shape)
    if real_out:
        out = torch.empty(rows.shape, dtype=rdt, device=x.device)
        work = torch.empty(rows.shape, dtype=cdt, device=x.device) if m > 12 else None
    else:
        out = torch.empty(rows.shape, dtype=cdt, device=x.device)
        work = None
    N.call("fgp_ifftbr_c64" if sp else "fgp_ifftbr", N.ptr(rows), bs, N.ptr(out), int(real_out), N.ptr(work),
           rows.size(0), m, int(stable), _stream(x))
    return out.reshape(shape)


def ifftbr_real_rf(x, f, n=None):
    """Re ifftbr(x * f) along the last dim for complex128 x [*, n] and REAL factor rows f (float64, one row or
    one per row of x), 2^17 <= n <= 2^24, at half length (fgp_ifftbr_real_rf): the coefficient solve
    ift(A * ytilde).real of gram_matrix_solve (util.py:341-343) with the spectral path's real A.  x must be
    Hermitian along the last dim (ft of real data, as ytilde) and f even (as A): only k <= n/2 are read -- so
    x may also be just that half, [*, n/2 + 1] (fftbr_real_half), with n given."""
    require_device(x, "ifftbr_real_rf")
    half = n is not None and x.shape[-1] == n // 2 + 1
    n = x.shape[-1] if n is None else int(n)
    m = log2_exact(n)
    assert 17 <= m <= 24, "ifftbr_real_rf needs 2^17 <= n <= 2^24"
    x = x.to(torch.complex128)
    rows, bs = _as_rows(x)
    f2 = resolved(f.to(device=x.device, dtype=torch.float64)).reshape(-1, n).contiguous()
    assert f2.size(0) in (1, rows.size(0)), "one factor row, or one per row of x"
    out = torch.empty((rows.size(0), n), dtype=torch.float64, device=x.device)
    work = torch.empty((rows.size(0), n), dtype=torch.complex128, device=x.device)
    N.call("fgp_ifftbr_real_rf", N.ptr(rows), bs, N.ptr(f2), 0 if f2.size(0) == 1 else n, N.ptr(out), n, N.ptr(work),
           rows.size(0), m, _stream(x))
    return out.reshape(x.shape[:-1] + (n,)) if half else out.reshape(x.shape)


def fwht_raw(x, stable=True):
    """Orthonormal Sylvester FWHT along the last dim (fgp_fwht, or fgp_fwht_f32 for float32 input)."""
    require_device(x, "fwht")
    if x.is_complex():
        return torch.complex(fwht_raw(x.real, stable), fwht_raw(x.imag, stable))
    sp = _single(x)
    rdt = torch.float32 if sp else torch.float64
    x = x.to(rdt)
    shape = x.shape
    m = log2_exact(shape[-1])
    rows, bs = _as_rows(x)
    out = torch.empty(rows.shape, dtype=rdt, device=x.device)
    N.call("fgp_fwht_f32" if sp else "fgp_fwht", N.ptr(rows), bs, N.ptr(out), rows.size(0), m, int(stable),
           _stream(x))
    return out.reshape(shape)


def sum_sq(x, G=1):
    """Y[g, k] = sum_r |x[r G + g, k]|^2 (fp64) over rows x [R G, n] (float64 / complex128 / float32 /
    complex64) -> [G, n] (fgp_sum_sq: the MLL data term of outputs sharing eigen-problem g)."""
    require_device(x, "sum_sq")
    n = x.shape[-1]
    rows, bs = _as_rows(x)
    assert rows.size(0) % G == 0
    kind = {torch.float64: 0, torch.complex128: 1, torch.float32: 2, torch.complex64: 3}[rows.dtype]
    out = torch.empty((G, n), dtype=torch.float64, device=x.device)
    N.call("fgp_sum_sq", N.ptr(rows), bs, kind, rows.size(0) // G, G, n, N.ptr(out), _stream(x))
    return out


def inverse_mul(family, x, f, real_out=False, stable=True):
    """inverse(x * f) along the last dim in one call (fgp_ifftbr_mul): ifftbr for lattices (real_out:
    the real part, gram_matrix_solve's .real, util.py:341-343), fwht for nets.  f [*, n] broadcasts
    against x [*, n] when it is one row, or matches x's rows; else the product is formed first."""
    require_device(x, "inverse_mul")
    sp = _single(x)
    n = x.shape[-1]
    m = log2_exact(n)
    if family == LATTICE:
        cdt = torch.complex64 if sp else torch.complex128
        x = x.to(cdt)
        f = f.to(cdt)
    else:
        rdt = torch.float32 if sp else torch.float64
        if x.is_complex() or f.is_complex():
            return fwht_raw(x * f, stable)
        x = x.to(rdt)
        f = f.to(rdt)
    rows, bs = _as_rows(x)
    f2 = resolved(f).reshape(-1, n)
    if f2.size(0) == 1:
        fbs = 0
    elif tuple(f.shape) == tuple(x.shape):
        fbs = n
    else:
        prod = x * f
        return ifftbr_raw(prod, stable, real_out) if family == LATTICE else fwht_raw(prod, stable)
    f2 = f2.contiguous()
    if family == LATTICE and real_out and stable and not sp and 17 <= m <= 24 and rows_ok_env():
        # Re ift(x * f) at half length (fgp_ifftbr_real, the product fused into the column loads)
        out = torch.empty(rows.shape, dtype=torch.float64, device=x.device)
        work = torch.empty(rows.shape, dtype=rows.dtype, device=x.device)
        N.call("fgp_ifftbr_real", N.ptr(rows), bs, N.ptr(f2), fbs, N.ptr(out), n, N.ptr(work), rows.size(0), m,
               _stream(x))
        return out.reshape(x.shape)
    if family == LATTICE:
        odt = (torch.float32 if sp else torch.float64) if real_out else rows.dtype
        out = torch.empty(rows.shape, dtype=odt, device=x.device)
        work = torch.empty(rows.shape, dtype=rows.dtype, device=x.device) if (real_out and m > 12) else None
    else:
        out = torch.empty(rows.shape, dtype=rows.dtype, device=x.device)
        work = None
    N.call("fgp_ifftbr_mul", int(family), int(sp), N.ptr(rows), bs, N.ptr(f2), fbs, N.ptr(out),
           int(bool(real_out) and family == LATTICE), N.ptr(work), rows.size(0), m, int(stable), _stream(x))
    shape = x.shape if not (real_out and family == LATTICE) else x.shape
    return out.reshape(shape)


class _FFTBR(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stable):
        ctx.real_in = not x.is_complex()
        ctx.stable = stable
        return fftbr_raw(x, stable)

    @staticmethod
    def backward(ctx, g):
        # y = A x  =>  dL/dx = A^H g (real part for a real x); A^H = ifftbr
        return ifftbr_raw(g, ctx.stable, real_out=ctx.real_in), None


class _IFFTBR(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stable):
        ctx.real_in = not x.is_complex()
        ctx.stable = stable
        return ifftbr_raw(x, stable)

    @staticmethod
    def backward(ctx, g):
        gx = fftbr_raw(g, ctx.stable)
        return (gx.real.contiguous() if ctx.real_in else gx), None


class _FWHT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stable):
        ctx.stable = stable
        return fwht_raw(x, stable)

    @staticmethod
    def backward(ctx, g):
        return fwht_raw(g, ctx.stable), None


def _graph_wanted(x):
    # (no autograd node when nothing needs one: the Function's bookkeeping is most of a small transform's host time)
    return torch.is_grad_enabled() and x.requires_grad


def fftbr(x, stable=False):
    """Drop-in for qmcpy.fftbr_torch (stable=False) or AbstractFastGP.ft on lattices (stable=True)."""
    return _FFTBR.apply(x, stable) if _graph_wanted(x) else fftbr_raw(x, stable)


def ifftbr(x, stable=False):
    """Drop-in for qmcpy.ifftbr_torch (stable=False) or AbstractFastGP.ift on lattices (stable=True)."""
    return _IFFTBR.apply(x, stable) if _graph_wanted(x) else ifftbr_raw(x, stable)


def fwht(x, stable=False):
    """Drop-in for qmcpy.fwht_torch (stable=False) or AbstractFastGP.ft/ift on nets (stable=True)."""
    return _FWHT.apply(x, stable) if _graph_wanted(x) else fwht_raw(x, stable)


# ------------------------------------------------------------------------------------- kernel parts
def lattice_coefficient(alpha):
    """(-1)^(alpha+1) (2 pi)^(2 alpha) / (2 alpha)!  evaluated exactly as fast_gp_lattice.py:272."""
    return _lattice_coefficient(int(alpha))


@functools.lru_cache(maxsize=None)
def _lattice_coefficient(alpha):
    order = torch.tensor(2 * alpha, dtype=torch.int64)
    return ((-1) ** (alpha + 1) * torch.exp(2 * alpha * math.log(2 * math.pi) - torch.lgamma(order + 1.0))).item()


def lattice_parts(x, z, alphas, out=None):
    """parts[j, i] = c_j B_{2 alpha_j}((x[i, j] - z[j]) % 1)  -> [d, n] (fast_gp_lattice.py:263-273)."""
    require_device(x, "lattice_parts")
    x = x.to(torch.float64)
    if x.stride(-1) != 1:
        x = x.contiguous()
    z = z.to(torch.float64).contiguous()
    n, d = x.shape
    if out is None:
        out = torch.empty((d, n), dtype=torch.float64, device=x.device)
    assert out.shape == (d, n) and out.is_contiguous() and out.dtype == torch.float64
    N.call("fgp_lattice_parts", N.ptr(x), x.stride(0), N.ptr(z), n, d, N.int_array([2 * a for a in alphas]),
           N.double_array([lattice_coefficient(a) for a in alphas]), N.ptr(out), _stream(x))
    return out


def lattice_points(z, shift, n_min, n_max, device=None):
    """Natural-order rank-1 lattice points [n_max - n_min, d] generated on the device (fgp_lattice_points),
    bit-identical to seqs.Lattice(n_min, n_max).  z: [d] ints; shift: [d] floats in [0, 1)."""
    shift = torch.as_tensor(shift, dtype=torch.float64, device=device)
    require_device(shift, "lattice_points")
    shift = shift.contiguous()
    d = shift.numel()
    x = torch.empty((n_max - n_min, d), dtype=torch.float64, device=shift.device)
    N.call("fgp_lattice_points", N.int64_array(z), N.ptr(shift), int(n_min), int(n_max), d, N.ptr(x), _stream(shift))
    return x


def net_points(C, shift, t, n_min, n_max, device):
    """Natural-order digital net points on the device (fgp_net_points), bit-identical to
    seqs.DigitalNetB2: (x [n, d] float64, xb [n, d] int64).  C: [d, mcols] t-bit ints, shift: [d]."""
    C = torch.as_tensor(np.asarray(C, dtype=np.uint64).astype(np.int64)).to(device).contiguous()
    sh = torch.as_tensor(np.asarray(shift, dtype=np.uint64).astype(np.int64)).to(device).contiguous()
    require_device(C, "net_points")
    d, mcols = C.shape
    xb = torch.empty((n_max - n_min, d), dtype=torch.int64, device=C.device)
    x = torch.empty((n_max - n_min, d), dtype=torch.float64, device=C.device)
    N.call("fgp_net_points", N.ptr(C), mcols, N.ptr(sh), int(n_min), int(n_max), d, int(t), N.ptr(xb), N.ptr(x),
           _stream(C))
    return x, xb


def lattice_parts_gen(z, shift, alphas, n):
    """The lattice parts [d, n] exactly as the FGP_PARTS_LATTICE fit kernels regenerate them
    (fgp_lattice_parts_gen); shift: device [d] (= x[0])."""
    require_device(shift, "lattice_parts_gen")
    shift = shift.to(torch.float64).reshape(-1).contiguous()
    d = shift.numel()
    assert len(set(int(a) for a in alphas)) == 1, "one smoothness for every dimension"
    parts = torch.empty((d, n), dtype=torch.float64, device=shift.device)
    N.call("fgp_lattice_parts_gen", N.int64_array(z), N.ptr(shift), log2_exact(n), d, 2 * int(alphas[0]),
           N.double_array([lattice_coefficient(a) for a in alphas]), N.ptr(parts), _stream(shift))
    return parts


def net_parts(xb, z, t, out=None, alphas=None):
    """Walsh parts of order alphas[j] (1..4, default 1) for delta = xb XOR z -> [d, n]
    (fast_gp_digital_net_b2.py:274-301; see fgp_net_parts)."""
    require_device(xb, "net_parts")
    xb = xb.to(torch.int64)
    if xb.stride(-1) != 1:
        xb = xb.contiguous()
    z = z.to(torch.int64).contiguous()
    n, d = xb.shape
    if out is None:
        out = torch.empty((d, n), dtype=torch.float64, device=xb.device)
    assert out.shape == (d, n) and out.is_contiguous() and out.dtype == torch.float64
    order = N.int_array([int(a) for a in alphas]) if alphas is not None else None
    N.call("fgp_net_parts", N.ptr(xb), xb.stride(0), N.ptr(z), n, d, int(t), order, N.ptr(out), _stream(xb))
    return out


# ------------------------------------------------------------------------------------- prediction
def _pred_args(family, alphas, d):
    if family == LATTICE:
        return N.int_array([2 * a for a in alphas]), N.double_array([lattice_coefficient(a) for a in alphas])
    return N.int_array([int(a) for a in alphas] if alphas is not None else [1] * d), N.double_array([0.0] * d)


def post_mean_chunk(n, Nt, target_wg=1024):
    """Training points per fgp_post_mean workgroup: 1024, or fewer (down to 32, powers of two) so that the
    launch (ceil(n / chunk) x ceil(N / 256) workgroups) has about `target_wg` workgroups -- 4 per CU; at
    n = 2^16 and N = 256, 1024 points per workgroup would leave 3/4 of the chip idle."""
    tiles = max(1, (Nt + 255) // 256)
    chunk = 1024
    while chunk > 32 and ((n + chunk - 1) // chunk) * tiles < target_wg:
        chunk //= 2
    return chunk


def post_mean_matfree(family, xt, z_dn, hyp, coeffs, alphas=None, tbits=0, chunk=None):
    """out[b, t] = sum_i K_{b mod Gk}(xt[t], z[:, i]) coeffs[b, i] -> [B, N] (see fgp_post_mean).

    xt [N, d] float64, z_dn [d, n] (float64 lattice / int64 net), hyp [Gk, 1 + d] (scale, lengthscales),
    coeffs [B, n]; chunk = training points per workgroup (default: post_mean_chunk)."""
    require_device(xt, "post_mean")
    xt = xt.to(torch.float64).contiguous()
    Nt, d = xt.shape
    n = z_dn.shape[1]
    hyp = hyp.to(torch.float64).contiguous()
    Gk = hyp.shape[0]
    B = coeffs.shape[0]
    if Gk == 1 and B >= GEMM_MIN_OUTPUTS:
        return post_mean_gemm(family, xt, z_dn, hyp, coeffs, alphas=alphas, tbits=tbits)
    coeffs = coeffs.to(torch.float64)
    if coeffs.stride(-1) != 1:
        coeffs = coeffs.contiguous()
    out = torch.empty((B, Nt), dtype=torch.float64, device=xt.device)
    order, coef = _pred_args(family, alphas, d)
    if Gk == B and B > 4:
        # every output with its own hyper-parameters (C5 per-output): ONE launch over the blocks of 4 outputs
        # (fgp_post_mean, ABI 16) instead of one per block -- no launch gaps, the rounds of resident workgroups filled
        if chunk is None:
            chunk = post_mean_chunk(n, Nt * (B // 4))
        nchunks = (n + chunk - 1) // chunk
        work = torch.empty((nchunks * B * Nt,), dtype=torch.float64, device=xt.device)
        hyp_c = hyp.contiguous()
        N.call("fgp_post_mean", family, N.ptr(xt), Nt, N.ptr(z_dn), n, d, int(tbits), order, coef, N.ptr(hyp_c), B,
               N.ptr(coeffs), coeffs.stride(0), B, N.ptr(out), Nt, N.ptr(work), chunk, _stream(xt))
        return out
    if chunk is None:
        chunk = post_mean_chunk(n, Nt)
    nchunks = (n + chunk - 1) // chunk
    work_all = torch.empty((nchunks * min(B, 4) * Nt,), dtype=torch.float64, device=xt.device)
    for b0 in range(0, B, 4):
        b1 = min(B, b0 + 4)
        if Gk == 1:
            hyp_b = hyp
        elif Gk == B:
            hyp_b = hyp[b0:b1]        # a view: no gather launch per block of 4 outputs
        else:
            hyp_b = hyp[torch.arange(b0, b1, device=hyp.device) % Gk]
        work = work_all[:nchunks * (b1 - b0) * Nt]
        cb = coeffs[b0:b1]
        N.call("fgp_post_mean", family, N.ptr(xt), Nt, N.ptr(z_dn), n, d, int(tbits), order, coef, N.ptr(hyp_b),
               hyp_b.shape[0], N.ptr(cb), cb.stride(0) if cb.shape[0] > 1 else n, b1 - b0, N.ptr(out[b0:b1]),
               Nt, N.ptr(work), chunk, _stream(xt))
    return out


# outputs sharing one kernel from which the posterior mean is a GEMM (kernel rows + rocBLAS)
GEMM_MIN_OUTPUTS = 8
GEMM_ROWS_BYTES = 1 << 28          # kernel-row block materialised per GEMM (256 MB)


def post_mean_gemm(family, xt, z_dn, hyp, coeffs, alphas=None, tbits=0):
    """Posterior mean of B outputs sharing hyper-parameters (BASELINE config C5: shape_batch = [B],
    shape_scale = [1]): out = coeffs @ K(xt, z)^T, [B, n] x [n, N] -- GEMM-shaped, so the kernel rows
    K(xt, z) are generated by fgp_kernel_rows in blocks of test points and contracted by the library
    GEMM (rocBLAS / hipBLASLt through torch.matmul, FP64 MFMA) instead of re-evaluating the kernel for
    every output (abstract_gp.py:375-377: kmat [N, n] einsum coeffs).  fp64 throughout: the mean is
    a heavily cancelling sum of K(x, z_i) c_i with |c| ~ |y| / noise, which an fp32 contraction does
    not resolve."""
    Nt, d = xt.shape
    n = z_dn.shape[1]
    B = coeffs.shape[0]
    cdt = torch.float64
    coeffs = coeffs.to(cdt)
    if coeffs.stride(-1) != 1:
        coeffs = coeffs.contiguous()
    out = torch.empty((B, Nt), dtype=torch.float64, device=xt.device)
    step = max(1, min(Nt, GEMM_ROWS_BYTES // (8 * n)))
    for t0 in range(0, Nt, step):
        t1 = min(Nt, t0 + step)
        rows = kernel_rows(family, xt[t0:t1], z_dn, hyp, alphas=alphas, tbits=tbits)[0]   # [Nc, n]
        out[:, t0:t1] = torch.matmul(coeffs, rows.to(cdt).T)
    return out


def kernel_rows(family, xt, z_dn, hyp, alphas=None, tbits=0):
    """rows[g, t, i] = K_g(xt[t], z[:, i]) -> [Gk, N, n]."""
    require_device(xt, "kernel_rows")
    xt = xt.to(torch.float64).contiguous()
    Nt, d = xt.shape
    n = z_dn.shape[1]
    hyp = hyp.to(torch.float64).contiguous()
    Gk = hyp.shape[0]
    rows = torch.empty((Gk, Nt, n), dtype=torch.float64, device=xt.device)
    order, coef = _pred_args(family, alphas, d)
    for t0 in range(0, Nt, 65535):
        t1 = min(Nt, t0 + 65535)
        sub = torch.empty((Gk, t1 - t0, n), dtype=torch.float64, device=xt.device) if Nt > 65535 else rows
        N.call("fgp_kernel_rows", family, N.ptr(xt[t0:t1]), t1 - t0, N.ptr(z_dn), n, d, int(tbits), order, coef,
               N.ptr(hyp), Gk, N.ptr(sub), _stream(xt))
        if sub is not rows:
            rows[:, t0:t1] = sub
    return rows


def post_var_quadform(family, xt, z_dn, hyp, wa, alphas=None, tbits=0):
    """q[t] = sum_k wa[k] |ft(K(xt[t], z))_k|^2 (fgp_post_var_qf); hyp: device [1 + d] (scale, l_1..l_d)."""
    require_device(xt, "post_var_quadform")
    Nt, d = xt.shape
    n = z_dn.shape[1]
    m = log2_exact(n)
    cdt = torch.complex128 if family == LATTICE else torch.float64
    work = torch.empty((Nt, n), dtype=cdt, device=xt.device)
    partial = torch.empty((Nt, n >> 12), dtype=torch.float64, device=xt.device)
    out = torch.empty(Nt, dtype=torch.float64, device=xt.device)
    order, coef = _pred_args(family, alphas, d)
    N.call("fgp_post_var_qf", family, N.ptr(xt), Nt, N.ptr(z_dn), m, d, int(tbits), order, coef,
           N.ptr(hyp.to(torch.float64).contiguous()), N.ptr(wa), N.ptr(work), N.ptr(partial), N.ptr(out), _stream(xt))
    return out


def double_update(family, prev, nxt):
    """ft of 2n values from ft of the first n (prev [..., n]) and of the next n (nxt [..., n]): one DIT
    stage (fgp_double_update; _LamCaches / _YtildeCache doubling, util.py:113-132,173-178)."""
    require_device(prev, "double_update")
    n = prev.shape[-1]
    m = log2_exact(n)
    dt = torch.complex128 if family == LATTICE else torch.float64
    p, ps = _as_rows(prev.to(dt))
    q, qs = _as_rows(nxt.to(dt).expand(prev.shape))
    out = torch.empty((p.shape[0], 2 * n), dtype=dt, device=prev.device)
    N.call("fgp_double_update", int(family), N.ptr(p), ps, N.ptr(q), qs, p.shape[0], m, N.ptr(out), 2 * n,
           _stream(prev))
    return out.reshape(tuple(prev.shape[:-1]) + (2 * n,))


# ------------------------------------------------------------------------------------- multitask
def mt_layout(ns_sorted):
    """fgp_mt_layout of the active tasks (n > 0, sorted by n descending)."""
    ns = [int(v) for v in ns_sorted]
    assert 1 <= len(ns) <= N.MT_MAX_TASKS, "multitask: %d active tasks (at most %d)" % (len(ns), N.MT_MAX_TASKS)
    lay = N.MtLayout()
    lay.T = len(ns)
    for k, v in enumerate(ns):
        lay.n[k] = v
    return lay


_MT_SPEC = {}


def mt_parts(family, x, z, order, coef, add, tbits=0, zip_pairs=False):
    """Derivative kernel parts (fgp_mt_parts): x [N, d], z [M, d] (float64 lattice / int64 net points);
    order / coef / add [P, d] host lists -> [N, M, P, d] (or [N, P, d] with zip_pairs, N == M)."""
    require_device(x, "mt_parts")
    dt = torch.float64 if family == LATTICE else torch.int64
    x = x.to(dt)
    z = z.to(dt)
    x = x if x.stride(-1) == 1 else x.contiguous()
    z = z if z.stride(-1) == 1 else z.contiguous()
    Nx, d = x.shape
    M = z.shape[0]
    P = len(order)
    dev = x.device
    # the [P, d] spec arrays on the device, made once per spec (a host list -> device tensor is a blocking copy)
    key = (str(dev), int(family), tuple(map(tuple, order)), tuple(map(tuple, coef)), tuple(map(tuple, add)))
    spec = _MT_SPEC.get(key)
    if spec is None:
        spec = (torch.tensor(order, dtype=torch.int32, device=dev).reshape(P, d).contiguous(),
                torch.tensor(coef, dtype=torch.float64, device=dev).reshape(P, d).contiguous(),
                torch.tensor(add, dtype=torch.float64, device=dev).reshape(P, d).contiguous())
        if len(_MT_SPEC) > 256:
            _MT_SPEC.clear()
        _MT_SPEC[key] = spec
    o, c, a = spec
    shape = (Nx, P, d) if zip_pairs else (Nx, M, P, d)
    out = torch.empty(shape, dtype=torch.float64, device=dev)
    N.call("fgp_mt_parts", int(family), N.ptr(x), x.stride(0) if Nx > 1 else d, Nx, N.ptr(z),
           z.stride(0) if M > 1 else d, M, int(bool(zip_pairs)), d, P, N.ptr(o), N.ptr(c), N.ptr(a), int(tbits),
           N.ptr(out), _stream(x))
    return out


def mt_factor(lay, lams):
    """Structured LDL^H of G problems' Gram blocks (fgp_mt_factor): lams [G, L] complex128 ->
    (factor [G, L], logdet per frequency class [G, nmin], info [1] int32 device flag)."""
    require_device(lams, "mt_factor")
    lams = resolved(lams.to(torch.complex128)).contiguous()
    G = lams.shape[0]
    nmin = int(lay.n[lay.T - 1])
    fac = torch.empty_like(lams)
    ld = torch.empty((G, nmin), dtype=torch.float64, device=lams.device)
    info = torch.zeros(1, dtype=torch.int32, device=lams.device)
    N.call("fgp_mt_factor", N.byref_layout(lay), N.ptr(lams), G, N.ptr(fac), N.ptr(ld), N.ptr(info), _stream(lams))
    return fac, ld, info


def mt_solve(lay, fac, v):
    """out[b] = Lambda_{b mod G}^-1 v[b] (fgp_mt_solve), v [B, R nmin] complex128."""
    require_device(v, "mt_solve")
    v = resolved(v.to(torch.complex128))
    v = v if v.stride(-1) == 1 and (v.shape[0] <= 1 or v.stride(0) >= v.shape[1]) else v.contiguous()
    B = v.shape[0]
    out = torch.empty((B, v.shape[1]), dtype=torch.complex128, device=v.device)
    N.call("fgp_mt_solve", N.byref_layout(lay), N.ptr(fac), fac.shape[0], N.ptr(v), v.stride(0) if B > 1 else v.shape[1],
           B, N.ptr(out), _stream(v))
    return out


def mt_selinv(lay, fac):
    """Entries of the inverse on the coupling pattern (fgp_mt_selinv) -> [G, L]."""
    out = torch.empty_like(fac)
    N.call("fgp_mt_selinv", N.byref_layout(lay), N.ptr(fac), fac.shape[0], N.ptr(out), _stream(fac))
    return out


class _MtMLL(torch.autograd.Function):
    """(norm_b = Re(y_b^H Lambda^-1 y_b), logdet_g) of packed lams [G, L] and tilde data Y [B, R nmin]
    (util.py:364-370 with the block inverse of util.py:275-337); backward by fgp_mt_selinv +
    fgp_mt_mll_grad (gradient w.r.t. the lams only; the data carry none)."""

    @staticmethod
    def forward(ctx, lams, Y, lay):
        fac, ld, _ = mt_factor(lay, lams)
        z = mt_solve(lay, fac, Y)
        norm = (Y.conj() * z).real.sum(-1)
        ctx.lay = lay
        ctx.save_for_backward(fac, z)
        return norm, ld.sum(-1)

    @staticmethod
    def backward(ctx, gn, gl):
        fac, z = ctx.saved_tensors
        lay = ctx.lay
        G, B = fac.shape[0], z.shape[0]
        zinv = mt_selinv(lay, fac)
        gn = (gn if gn is not None else torch.zeros(B, device=z.device, dtype=torch.float64)).to(torch.float64).contiguous()
        gl = (gl if gl is not None else torch.zeros(G, device=z.device, dtype=torch.float64)).to(torch.float64).contiguous()
        glp = torch.empty_like(fac)
        N.call("fgp_mt_mll_grad", N.byref_layout(lay), N.ptr(zinv), N.ptr(z), N.ptr(gn), N.ptr(gl), B, G, N.ptr(glp),
               _stream(z))
        return glp, None, None


def mt_mll_terms(lay, lams, Y):
    """Differentiable (norm [B], logdet [G]) for the multitask MLL (HIP factor / solve / gradient)."""
    return _MtMLL.apply(resolved(lams.to(torch.complex128)).contiguous(),
                        resolved(Y.to(torch.complex128)).contiguous(), lay)
