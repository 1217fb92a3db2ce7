"""GPU parity of the spectral fit path (part-product spectra, include/fgp_hip.h ABI 11).

lambda = ft(k1) with k1 = scale prod_j (1 + l_j parts_j) (abstract_fast_gp.py:181-191, util.py:95-112) is,
by linearity of ft, scale sum_S l^S Phi_S with Phi_S = ft(prod_{j in S} parts_j).  Checked here:
  * fgp_spec_basis against the oracle's stable transforms of the same products (fftbr real part k <= n/2
    for lattices, fwht for nets): 1e-13 (1 + m) relative, the transform tolerance of test_gpu_transforms.py;
  * lambda from the spectra (fgp_nll_lam) against the oracle's ft(k1): 1e-12 relative (test_gpu_gp.py);
  * the one-kernel iteration's loss and gradient (fgp_nll_fwd / fgp_fit_step on a spectral desc) against
    the oracle's MLL + autograd: 2e-7 relative (the lattice MLL's backend spread x 5, test_gpu_gp.py);
  * fits by the spectral path and by the transform kernels (FGP_FIT_PATH) against each other: parameters
    1e-9 (Rprop takes only gradient signs), loss histories 2e-6 relative (losses up to 1e9 next to the
    nugget, the oracle tests' 2e-7 scale), posterior means 1e-7;
  * batched problems sharing one set of spectra (per-problem hyper-parameters, the C4 shifts) equal
    individual fits bit for bit.
"""
import math

import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from fastgaussianprocesses_amd.fit_engine import fused_lam, mll_constant, spec_basis, spec_dense, spectral_wanted
from oracle import fgp_oracle as O
from tests.gpu_fixtures import DEV, rel_err

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)


def _gp(family, d, m, seed=7, **kw):
    if family == "lattice":
        gp = F.FastGPLattice(F.Lattice(d, seed=seed), device=DEV, **kw)
    else:
        gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=seed), device=DEV, **kw)
    x = gp.get_x_next(2 ** m)
    y = O.f_ackley(x.cpu())
    if "shape_batch" in kw:
        B = int(np.prod(kw["shape_batch"]))
        y = y[None, :] * (1 + torch.arange(B, dtype=torch.float64)[:, None] / B)
    gp.add_y_next(y.to(DEV))
    return gp, x.cpu(), y


def _oracle(family, gp, x, y):
    xb = gp.get_xb().cpu() if family == "net" else None
    return O.OracleFastGP(family, x, xb, y, alpha=gp._alphas[0], t=getattr(gp, "t", None))


@pytest.mark.parametrize("family", ["lattice", "net"])
@pytest.mark.parametrize("m,d", [(4, 1), (8, 3), (12, 5), (16, 3), (17, 2), (18, 5)])
def test_basis_matches_oracle_transforms(family, m, d):
    gp, _, _ = _gp(family, d, m)
    n = 2 ** m
    fam = gp._FAMILY
    parts = gp._k1parts(n)
    raw = spec_basis(fam, parts, n).cpu()
    K = n // 2 + 1 if family == "lattice" else n
    Q = (K + 63) // 64
    assert raw.shape == (Q, 2 ** d, 64)
    full = raw.movedim(0, 1).reshape(2 ** d, Q * 64)
    assert not full[:, K:].any()                      # zero padding past K
    basis = spec_dense(raw, fam, n)
    pc = parts.cpu()
    tr = O.fftbr if family == "lattice" else O.fwht
    for S in range(2 ** d):
        b = torch.ones(n)
        for j in range(d):
            if (S >> j) & 1:
                b = b * pc[j]
        ref = O.ft_stable(b, tr)
        ref = ref.real[:K] if family == "lattice" else ref
        assert rel_err(basis[S, :K], ref) <= 1e-13 * (1 + m), (S, rel_err(basis[S, :K], ref))


@pytest.mark.parametrize("family", ["lattice", "net"])
@pytest.mark.parametrize("m,d", [(10, 2), (16, 3), (18, 5)])
def test_spectral_lam_loss_and_gradient_match_oracle(family, m, d):
    gp, x, y = _gp(family, d, m)
    n = 2 ** m
    g = torch.Generator().manual_seed(m + d)
    ls = torch.exp(torch.randn(d, generator=g))          # off the default point: every subset weighted
    with torch.no_grad():
        gp.raw_lengthscales.copy_(torch.log(ls).to(DEV))
        gp.raw_scale.fill_(math.log(1.7))
    o = _oracle(family, gp, x, y)
    with torch.no_grad():
        o.raw_lengthscales.copy_(torch.log(ls))
        o.raw_scale.fill_(math.log(1.7))
    basis = spec_basis(gp._FAMILY, gp._k1parts(n), n)
    lam = fused_lam(gp._FAMILY, None, gp.raw_scale.detach().reshape(-1), gp.raw_lengthscales.detach().reshape(1, -1),
                    gp.raw_noise.detach().reshape(-1), 1, n=n, basis=basis)
    olam = o.lam().detach()
    assert rel_err(lam[0], olam) <= 1e-12
    eng = F.FusedMLL(gp._FAMILY, None, gp._ysq(*gp._problem_batch()), gp.raw_scale.detach().reshape(-1),
                     gp.raw_lengthscales.detach().reshape(1, -1), gp.raw_noise.detach().reshape(-1), logdet_weight=1.0,
                     mll_const=mll_constant(1, n), basis=basis)
    loss, t1, t2, grad = eng.evaluate()
    oloss, ot1, ot2 = o.mll_loss()
    gs, gl = torch.autograd.grad(oloss, [o.raw_scale, o.raw_lengthscales])
    assert rel_err(loss, oloss) <= 2e-7
    assert rel_err(t1, ot1) <= 2e-7
    assert rel_err(grad[:1], gs.reshape(-1)) <= 2e-7
    assert rel_err(grad[1:1 + d], gl.reshape(-1)) <= 2e-7


@pytest.mark.parametrize("family,m,d,kw", [("lattice", 12, 3, {}), ("lattice", 17, 5, {}), ("net", 14, 3, {}),
                                           ("lattice", 14, 2, dict(shape_batch=[3], shape_scale=[3, 1],
                                                                   shape_lengthscales=[3, 2]))])
def test_spectral_and_transform_fits_agree(family, m, d, kw, monkeypatch):
    res = {}
    for path in ("spectral", "transform"):
        monkeypatch.setenv("FGP_FIT_PATH", path)
        gp, _, _ = _gp(family, d, m, **kw)
        data = gp.fit(iterations=12, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=20)
        res[path] = (data["loss_hist"], torch.cat([gp.raw_scale.detach().reshape(-1), gp.raw_lengthscales.detach().reshape(-1)]).cpu(),
                     gp.post_mean(torch.rand((16, d), generator=torch.Generator().manual_seed(3)).to(DEV)).cpu())
    (la, pa, ma), (lb, pb, mb) = res["spectral"], res["transform"]
    assert float((pa - pb).abs().max()) <= 1e-9
    # the two paths round lambda differently; near the 1e-8 nugget the loss amplifies that to the level
    # the oracle tests allow (2e-7, test_gpu_gp.py), here on losses up to 1e9
    assert rel_err(la, lb) <= 2e-6
    assert rel_err(ma, mb) <= 1e-7


def test_spectral_batch_shares_one_basis_and_equals_individual_fits(monkeypatch):
    """The C4 shape (randomly shifted lattice GPs, one generating vector) at a small size: ONE set of
    spectra for the batch; batched per-problem fits equal each GP's own fit bit for bit."""
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    d, m = 5, 14
    def make():
        gps = []
        for seed in (11, 12, 13):
            gp = F.FastGPLattice(F.Lattice(d, seed=seed), device=DEV)
            x = gp.get_x_next(2 ** m)
            gp.add_y_next(O.f_ackley(x.cpu()).to(DEV))
            gps.append(gp)
        return gps
    gps = make()
    b = F.GPBatch(gps)
    b.set_data(torch.stack([gp._y[0] for gp in gps]))
    basis = b.basis()
    assert basis is not None and basis.shape == ((2 ** (m - 1) + 1 + 63) // 64, 2 ** d, 64)
    data = b.fit(iterations=8, stop_crit_wait_iterations=20, store_loss_hist=True)
    ind = make()
    for p, gp in enumerate(ind):
        dp = gp.fit(iterations=8, stop_crit_wait_iterations=20, store_loss_hist=True, verbose=0)
        assert torch.equal(dp["loss_hist"], data[p]["loss_hist"])
        assert torch.equal(gp.raw_lengthscales.detach(), gps[p].raw_lengthscales.detach().reshape(gp.raw_lengthscales.shape))


@pytest.mark.parametrize("m", [17, 20])
def test_spectral_coefficients_from_spectra(m):
    """GPBatch.coeffs on the spectral path (fgp_spec_inv_eig: A = 1/ev straight from the spectra, the product
    fused into the half-length inverse with real factor rows, fgp_ifftbr_real_rf) against the lambda route
    (fgp_nll_lam + fgp_inv_eig + fgp_ifftbr_real) and the oracle's K^-1 y (util.py:338-353)."""
    from fastgaussianprocesses_amd import ops
    d, P = 3, 3
    gps = [F.FastGPLattice(F.Lattice(d, seed=40 + p, randomize="SHIFT"), device=DEV) for p in range(P)]
    for p, gp in enumerate(gps):
        x = gp.get_x_next(2 ** m)
        gp.add_y_next(O.f_ackley(x.cpu()).to(DEV) * (1 + 0.1 * p))
        with torch.no_grad():
            gp.raw_lengthscales.add_(0.05 * p)
    b = F.GPBatch(gps)
    assert b.basis() is not None
    c = b.coeffs()
    wa = b._st["wa"]
    raw = b.raw()
    dl = b.dl
    lam = fused_lam(0, None, raw[:, 0], raw[:, 1:1 + dl], raw[:, 1 + dl], P, n=2 ** m, basis=b.basis())
    ev = math.sqrt(2 ** m) * lam.real + torch.exp(raw[:, 1 + dl])[:, None]
    assert rel_err(wa, 1.0 / ev) < 1e-14
    ref = ops.ifftbr_raw(b.ytilde() * (1.0 / ev), stable=True, real_out=True)
    assert rel_err(c, ref) < 1e-12
    # real factor rows: one shared row and per-row rows give Re ifftbr(x * f)
    assert rel_err(ops.ifftbr_real_rf(b.ytilde(), wa[:1]), ops.ifftbr_raw(b.ytilde() * wa[:1], True, True)) < 1e-13
    if m == 17:
        for p, gp in enumerate(gps):
            o = O.OracleFastGP("lattice", gp.get_x(0).cpu(), None, gp._y[0].cpu(), alpha=2)
            with torch.no_grad():
                o.raw_scale.copy_(gp.raw_scale.cpu())
                o.raw_lengthscales.copy_(gp.raw_lengthscales.cpu())
                o.raw_noise.copy_(gp.raw_noise.cpu())
            # coeffs = K^-1 y at cond(K) ~ n / noise: the 1e-5 of DESIGN.md section 1 (measured 1.8e-6)
            assert rel_err(c[p], o.coeffs().detach()) < 1e-5


@pytest.mark.parametrize("m,d,G", [(14, 3, 40), (17, 3, 16), (14, 5, 19), (12, 2, 9)])
def test_problem_slices_equal_per_wave_kernel(m, d, G, monkeypatch):
    """Many eigen-problems on one set of spectra (per-output hyper-parameters, shape_scale = [G, 1],
    docs/examples/batch_multitask/fgp_lattice.ipynb cell 6): the tile kernel over problem slices (G > 8:
    slices of 16 problems at d <= 3, 8 above; ragged last slice) against the per-wave kernel k_spec_iter
    (FGP_SPEC_TILE=0) -- the same per-block partials in the same order, so the fits agree to rounding of
    the fixed reduction (1e-13); parameters after 6 iterations to 1e-12; the spectral coefficients
    (fgp_spec_inv_eig + fgp_ifftbr_real_rf at m >= 17) against the lambda route to 1e-12."""
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    g = torch.Generator().manual_seed(G)
    ls0 = 0.3 * torch.randn((G, d), generator=g)
    res = {}
    for tile in ("1", "0"):
        monkeypatch.setenv("FGP_SPEC_TILE", tile)
        gp, _, _ = _gp("lattice", d, m, shape_batch=[G], shape_scale=[G, 1], shape_lengthscales=[G, d])
        with torch.no_grad():
            gp.raw_lengthscales.add_(ls0.to(DEV))
        data = gp.fit(iterations=6, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=20)
        with torch.no_grad():
            c = gp.coeffs.clone()
            if m >= 17:      # the spectral coefficient route against ift(ft(y) / ev).real (util.py:338-353)
                assert rel_err(c, gp._solve(gp._y[0], 2 ** m)) <= 1e-12
        res[tile] = (data["loss_hist"].cpu(), gp.raw_lengthscales.detach().cpu().clone(), c.cpu())
    (la, pa, ca), (lb, pb, cb) = res["1"], res["0"]
    assert rel_err(la, lb) <= 1e-13
    assert float((pa - pb).abs().max()) <= 1e-12
    assert rel_err(ca, cb) <= 1e-12


@pytest.mark.parametrize("m,d,G", [(14, 3, 40), (17, 2, 16), (15, 4, 20)])
def test_spectral_post_var_equals_per_row_transforms(m, d, G, monkeypatch):
    """Posterior variance of G problems on one point set (per-output hyper-parameters) from the row spectra
    of the test points (fgp_spec_post_var: ft(K_g(x_t, .)) = scale_g sum_S l_g^S Psi_S(t) by linearity, A
    from the fit's spectra) against one transform per (problem, test point) (fgp_post_var_batched,
    FGP_SPEC_POST_VAR=0): the quadratic forms agree to rounding; var = K(x,x) - qf is compared on the
    scale of K(x,x) (1e-10), as it cancels near the data.  Also at a future n = 2^(m+1)."""
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    g = torch.Generator().manual_seed(G + d)
    gp, _, _ = _gp("lattice", d, m, shape_batch=[G], shape_scale=[G, 1], shape_lengthscales=[G, d])
    with torch.no_grad():
        gp.raw_lengthscales.add_((0.3 * torch.randn((G, d), generator=g)).to(DEV))
        gp.raw_scale.add_((0.2 * torch.randn((G, 1), generator=g)).to(DEV))
        gp.raw_noise.fill_(math.log(1e-4))
    x = torch.rand((5, d), generator=g).to(DEV)
    kxx = gp._kdiag(x).detach().reshape(G, 1)
    for n in (None, 2 ** (m + 1)):
        monkeypatch.setenv("FGP_SPEC_POST_VAR", "1")
        gp._cache = {}
        v_spec = gp.post_var(x, n=n).reshape(G, -1)
        assert gp._post_var_spectral(x, n or 2 ** m, G) is not None
        monkeypatch.setenv("FGP_SPEC_POST_VAR", "0")
        gp._cache = {}
        v_row = gp.post_var(x, n=n).reshape(G, -1)
        assert float(((v_spec - v_row).abs() / kxx).max()) <= 1e-10
        assert bool((v_spec >= 0).all())


def test_spectral_post_var_slices_test_points(monkeypatch):
    """fgp_spec_post_var takes at most 4096 test points per call and the row products / spectra are sized per
    slice: slices of 2 points (forced through fast_gp.SPEC_POST_VAR_MAX_N) give the unsliced
    result bit for bit, and the per-row transforms (FGP_SPEC_POST_VAR=0) to 1e-10 K(x,x)."""
    from fastgaussianprocesses_amd import fast_gp
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    G, d, m = 16, 2, 17
    gp, _, _ = _gp("lattice", d, m, shape_batch=[G], shape_scale=[G, 1], shape_lengthscales=[G, d])
    x = torch.rand((7, d), generator=torch.Generator().manual_seed(3)).to(DEV)
    whole = gp._post_var_spectral(x, 2 ** m, G)
    monkeypatch.setattr(fast_gp, "SPEC_POST_VAR_MAX_N", 2)
    sliced = gp._post_var_spectral(x, 2 ** m, G)
    assert torch.equal(whole, sliced)
    monkeypatch.setenv("FGP_SPEC_POST_VAR", "0")
    gp._cache = {}
    v_row = gp.post_var(x).reshape(G, -1)
    kxx = gp._kdiag(x).detach().reshape(G, 1)
    assert float(((sliced - v_row).abs() / kxx).max()) <= 1e-10


@pytest.mark.parametrize("m,rows", [(17, 3), (18, 2), (20, 1)])
def test_real_factor_inverse_reads_half_of_hermitian_input(m, rows):
    """fgp_ifftbr_real_rf (ABI 13) reads only k <= n/2 of its Hermitian input (ft of real data) and even
    factor rows: equal to the full-length Re ifftbr(x * f) (1e-13 relative), for one shared factor row and one
    row per input; the n - k half of the input is never read (poisoned with NaN here)."""
    from fastgaussianprocesses_amd import ops
    n = 2 ** m
    g = torch.Generator().manual_seed(m)
    y = torch.randn((rows, n), generator=g, dtype=torch.float64).to(DEV)
    x = ops.fftbr_raw(y, stable=True)
    h = torch.rand((rows, n), generator=g, dtype=torch.float64).to(DEV) + 0.5
    f = h + h[:, (-torch.arange(n, device=DEV)) % n]                    # even: f_{n-k} = f_k
    for fr in (f[:1], f):
        ref = ops.ifftbr_raw(x * fr, stable=True, real_out=True)
        xp = x.clone()
        xp[:, n // 2 + 1:] = float("nan")
        got = ops.ifftbr_real_rf(xp, fr)
        assert rel_err(got, ref) <= 1e-13


@pytest.mark.parametrize("family,m,d,wait", [("lattice", 16, 3, 60), ("net", 16, 3, 60), ("lattice", 10, 6, 10),
                                             ("net", 10, 2, 10), ("lattice", 12, 1, 4), ("lattice", 18, 3, 60),
                                             ("net", 17, 2, 10)])
@pytest.mark.parametrize("hists", [True, False])
def test_single_launch_fit_equals_launch_per_iteration(family, m, d, wait, hists, monkeypatch):
    """fgp_fit_persist (the whole fit of one small spectral problem in one launch: LDS-resident spectra, an
    in-kernel grid barrier per iteration, the early-stopping rule on the device) against the launch per
    iteration (FGP_FIT_PERSIST=0): the same iterations, loss history and fitted parameters bit for bit --
    with early stopping impossible (wait 60 > 50 iterations: C2 / C3's bench step) and possible; n = 2^17 / 2^18
    spread the spectra over 128 workgroups (the C5 shared-parameter fit's geometry).  Without histories the host
    restores the best iterate the kernel left in the engine's raw parameters (ABI 18) while the launch runs."""
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    out = {}
    for persist in ("1", "0"):
        monkeypatch.setenv("FGP_FIT_PERSIST", persist)
        gp, _, _ = _gp(family, d, m)
        assert gp._fused_engine(1, 0.1).persist_ok() == (persist == "1")
        data = gp.fit(iterations=50, store_hists=hists, verbose=0, stop_crit_wait_iterations=wait)
        out[persist] = (data, gp.raw_scale.detach().cpu().clone(), gp.raw_lengthscales.detach().cpu().clone())
    (a, sa, la), (b, sb, lb) = out["1"], out["0"]
    assert a["iterations"] == b["iterations"]
    if hists:
        assert torch.equal(a["loss_hist"], b["loss_hist"])
        assert torch.equal(a["lengthscales_hist"], b["lengthscales_hist"])
    assert torch.equal(sa, sb) and torch.equal(la, lb)


@pytest.mark.parametrize("hists", [True, False])
@pytest.mark.parametrize("family,wait", [("lattice", 60), ("net", 10)])
def test_single_launch_fit_barrier_give_up_falls_back(family, wait, hists, monkeypatch):
    """A give-up of fgp_fit_persist's in-kernel grid barrier (forced by the test hook fgp_set_persist_poll_max(0):
    every wait that does not find the grid complete gives up at once) is detected in the SAME fit call: the
    kernel leaves NaN parameters and history, the host reads the control word, restores the entry parameters and
    re-runs the fit on the launch per iteration -- the result equals the normal single-launch fit bit for bit,
    with early stopping impossible (C2's bench step) and possible."""
    from fastgaussianprocesses_amd import _native as N
    from fastgaussianprocesses_amd.fit_engine import FusedMLL
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    monkeypatch.setenv("FGP_FIT_PERSIST", "1")
    runs, fails = {}, []
    orig = FusedMLL.persist_result        # (the control word's read: in run_persist, or deferred after the restore)

    def spy(self, *a, **k):
        r = orig(self, *a, **k)
        fails.append(r is None)
        return r
    monkeypatch.setattr(FusedMLL, "persist_result", spy)
    for poll in (-1, 0):
        gp, _, _ = _gp(family, 3, 16)
        assert gp._fused_engine(1, 0.1).persist_workgroups() >= 2, "C2 / C3 run the single-launch fit over >= 2 workgroups"
        N.call("fgp_set_persist_poll_max", poll)
        try:
            data = gp.fit(iterations=50, store_hists=hists, verbose=0, stop_crit_wait_iterations=wait)
        finally:
            N.call("fgp_set_persist_poll_max", -1)
        runs[poll] = (data, gp.raw_scale.detach().cpu().clone(), gp.raw_lengthscales.detach().cpu().clone())
    assert fails == [False, True], fails
    (a, sa, la), (b, sb, lb) = runs[-1], runs[0]
    assert a["iterations"] == b["iterations"]
    if hists:
        assert torch.equal(a["loss_hist"], b["loss_hist"])
        assert torch.equal(a["lengthscales_hist"], b["lengthscales_hist"])
    assert torch.equal(sa, sb) and torch.equal(la, lb)
    assert bool(torch.isfinite(sb).all()) and bool(torch.isfinite(lb).all())


@pytest.mark.parametrize("m,d,alpha", [(17, 1, 2), (17, 5, 2), (18, 3, 1), (18, 6, 2), (17, 2, 4)])
def test_basis_from_generating_vector_equals_parts_array_basis(m, d, alpha):
    """fgp_spec_basis_gen (ABI 15: the lattice parts regenerated in the transform's row pass) against
    fgp_spec_basis of the fgp_lattice_parts_gen array: the same spectra bit for bit (so the batch / single
    GP fits that switched to it keep their trajectories), and the lengthscale-free subsets against the
    oracle's transform of the product of parts."""
    from fastgaussianprocesses_amd import ops
    from fastgaussianprocesses_amd.fit_engine import LatticePartsGen, spec_basis_gen
    n = 2 ** m
    rng = np.random.default_rng(m + d)
    z = [int(v) for v in (2 * rng.integers(1, 2 ** (m - 1), size=d) + 1)]
    shift = torch.rand((1, d), dtype=torch.float64, generator=torch.Generator().manual_seed(d)).to(DEV)
    gen = LatticePartsGen(z, [alpha] * d, shift)
    got = spec_basis_gen(gen, n, torch.device(DEV), force=True)
    assert got is not None
    ref = spec_basis(0, ops.lattice_parts_gen(gen.z, gen.shift[0], gen.alphas, n), n)
    assert got.shape == ref.shape
    assert torch.equal(got, ref)


@pytest.mark.parametrize("m", [17, 20])
def test_persistent_fit_launch_equals_launch_per_iteration(m, monkeypatch):
    """The persistent k_spec_tile (FGP_SPEC_PERSIST=1: every iteration of an fgp_fit_run call and the last step in
    ONE launch, the launch boundary replaced by a wait on the published group sums) against one launch per
    iteration: the bench's C4 batch (8 shifted lattice GPs, d = 5), loss histories and fitted parameters bit for
    bit; with the spectra built from the generating vector (FGP_SPEC_BASIS_GEN=1) as well."""
    import argparse
    import bench
    d, n, P = 5, 2 ** m, 8
    dev = torch.device(DEV, 0)
    g = torch.Generator().manual_seed(17)
    xm, xv = torch.rand((8, d), generator=g).to(dev), torch.rand((2, d), generator=g).to(dev)
    out = {}
    for persist, bgen in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("FGP_SPEC_PERSIST", persist)
        monkeypatch.setenv("FGP_SPEC_BASIS_GEN", bgen)
        sh = bench.Shifts(F, d, n, bench.shard_seeds(0, 1, P), dev)
        data, pm, pv = bench.step_batched(sh, argparse.Namespace(fit_iters=12), xm, xv, store_loss_hist=True)
        out[(persist, bgen)] = ([dd["loss_hist"] for dd in data], sh.batch.raw().cpu().clone(), pm.cpu(), pv.cpu())
    ref = out[("0", "0")]
    for key in (("1", "0"), ("1", "1")):
        got = out[key]
        assert all(torch.equal(a, b) for a, b in zip(got[0], ref[0])), key
        assert torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2]) and torch.equal(got[3], ref[3]), key
        assert torch.isfinite(got[1]).all()


def test_single_launch_fit_give_up_inside_replayed_graph_raises(monkeypatch):
    """A give-up of fgp_fit_persist inside a hipGraph replay (the bench's C2 / C3 lines replay captured fits, whose
    control word the capture cannot read) is counted by the library's sticky give-up count (fgp_persist_giveups, ABI
    17) and fit_engine.check_replayed_fits raises -- instead of the replay silently returning NaN parameters."""
    from fastgaussianprocesses_amd import _native as N
    from fastgaussianprocesses_amd import fit_engine as E
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    monkeypatch.setenv("FGP_FIT_PERSIST", "1")
    gp, _, _ = _gp("lattice", 3, 16)
    gp.fit(iterations=5, verbose=0, stop_crit_wait_iterations=60)          # spectra / ytilde cached, kernels loaded
    before = E.persist_giveups()
    E.check_replayed_fits(before)                                          # nothing since: no raise
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            gp.fit(iterations=50, verbose=0, stop_crit_wait_iterations=60)
            out = gp.raw_lengthscales.detach().clone()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all())
    E.check_replayed_fits(before)                                          # a good replay: no raise
    N.call("fgp_set_persist_poll_max", 0)
    try:
        g.replay()
        torch.cuda.synchronize()
    finally:
        N.call("fgp_set_persist_poll_max", -1)
    assert not bool(torch.isfinite(out).all())                             # what a replay leaves: NaN parameters
    with pytest.raises(RuntimeError, match="give-up"):
        E.check_replayed_fits(before)
    E.persist_giveups(reset=True)
    # (the captured engine, kept by fit_engine.cached_engine, still holds the failed replay's control word, which its
    # next eager fit would report: drop it, so later tests of the same geometry start clean)
    del g
    E._ENGINES.clear()


def _graph_stats():
    import ctypes
    from fastgaussianprocesses_amd import _native as N
    out = (ctypes.c_longlong * 3)()
    N.call("fgp_fit_graph_stats", out)
    return list(out)


@pytest.mark.parametrize("case", ["c4_batch", "c5_per_output", "c2_per_launch"])
def test_fit_run_graph_replay_is_bit_identical_to_eager_launches(case, monkeypatch):
    """fgp_fit_run replays its spectral launch sequence from a cached hipGraph (ABI 17): the fit through the graph --
    captured on the first call, replayed from the cache on the second -- equals the eager launch sequence
    (FGP_FIT_GRAPH=0) bit for bit: loss histories, fitted parameters.  C4's batch of shifts (k_spec_tile, the
    deferred step), C5 per-output (the sliced tile + k_spec_step_many) and C2 on the launch per iteration."""
    import bench
    dev = torch.device("cuda", 0)
    if case == "c2_per_launch":
        monkeypatch.setenv("FGP_FIT_PERSIST", "0")
    res = {}
    for mode in ("0", "1", "1"):
        monkeypatch.setenv("FGP_FIT_GRAPH", mode)
        s0 = _graph_stats()
        if case == "c4_batch":
            sh = bench.Shifts(F, 5, 2 ** 17, bench.shard_seeds(0, 1, 4), dev)
            sh.reset()
            data = sh.batch.fit(iterations=20, stop_crit_wait_iterations=21, store_loss_hist=True)
            lh = torch.stack([d["loss_hist"] for d in data])
            raw = sh.batch.raw().cpu().clone()
        else:
            if case == "c5_per_output":
                sg = bench.MultiOutputGP(F, 16, 3, 32, dev, per_output=True)
            else:
                sg = bench.SingleGP(F, "lattice", 16, 3, dev)
            sg.reset()
            data = sg.gp.fit(iterations=20, stop_crit_wait_iterations=21, verbose=0, store_loss_hist=True)
            lh = data["loss_hist"]
            raw = torch.cat([sg.gp.raw_scale.detach().reshape(-1), sg.gp.raw_lengthscales.detach().reshape(-1)]).cpu()
        s1 = _graph_stats()
        res.setdefault(mode, []).append((lh, raw, [b - a for a, b in zip(s0, s1)]))
    (lh0, raw0, st0), = res["0"]
    assert st0[0] == st0[1] == 0, st0                        # FGP_FIT_GRAPH=0: eager
    for lh, raw, st in res["1"]:
        assert torch.equal(lh, lh0) and torch.equal(raw, raw0)
        assert st[0] + st[1] >= 1, st                        # the graph ran


def test_fit_run_graph_cached_replay_equals_eager(monkeypatch):
    """The same engine run again (its buffers unmoved): fgp_fit_run_graph replays the executable graph it cached for
    this engine token -- bit-identical to the first (captured) run and to the eager sequence."""
    monkeypatch.setenv("FGP_FIT_PATH", "spectral")
    gp, _, _ = _gp("lattice", 3, 16)
    eng = gp._fused_engine(50, 0.1)
    raw0, prev0, step0 = eng.raw.clone(), eng.prev.clone(), eng.step.clone()
    out = []
    for r, mode in enumerate(("1", "1", "1", "0")):
        monkeypatch.setenv("FGP_FIT_GRAPH", mode)
        eng.raw.copy_(raw0)
        eng.prev.copy_(prev0)
        eng.step.copy_(step0)
        eng.loss_hist.zero_()
        s0 = _graph_stats()
        eng.run(0, 51, final_no_update=True)
        d = [b - a for a, b in zip(s0, _graph_stats())]
        out.append((eng.loss_hist[:51].cpu().clone(), eng.raw.cpu().clone()))
        assert d == ([0, 1, 0] if r == 0 else [1, 0, 0] if mode == "1" else [0, 0, 0]), (r, d)
    for lh, raw in out[1:]:
        assert torch.equal(lh, out[0][0]) and torch.equal(raw, out[0][1])
