"""Parity at the BASELINE.json configurations (C2: FastGPLattice n=2^16 d=3; C3: FastGPDigitalNetB2
n=2^16 d=3 with the reference's default alpha=2; C4: FastGPLattice n=2^20 d=5, the bench workload):
the drop-in classes on the GPU (fused fit kernels, matrix-free post_mean, Parseval post_var) against
the CPU oracle (oracle/fgp_oracle.py, the reference's op sequence in torch-CPU) on the same points and
data.  Tolerances as tests/test_gpu_gp.py: MLL trajectory 2e-7 relative (ill-conditioned at the
nugget), posterior mean 1e-7 relative, posterior variance 1e-8 K(x,x) absolute.
"""
import pytest
import torch

import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O
from tests.gpu_fixtures import DEV

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)


@pytest.mark.parametrize("family,m,d,its,npm,npv", [("lattice", 16, 3, 5, 32, 4), ("net", 16, 3, 5, 32, 4),
                                                    ("lattice", 20, 5, 3, 8, 2)])
def test_config_fit_and_predict_match_oracle(family, m, d, its, npm, npv):
    n = 2 ** m
    if family == "lattice":
        gp = F.FastGPLattice(F.Lattice(d, seed=7), device=DEV)
    else:
        gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=7), device=DEV)   # default alpha = 2
    x = gp.get_x_next(n)
    y = O.f_ackley(x.cpu())
    gp.add_y_next(y.to(DEV))
    data = gp.fit(iterations=its, store_hists=True, verbose=0, stop_crit_wait_iterations=its + 5)
    o = O.OracleFastGP(family, x.cpu(), gp.get_xb().cpu() if family == "net" else None, y,
                       alpha=gp._alphas[0], t=getattr(gp, "t", None))
    od = o.fit(iterations=its, stop_crit_wait_iterations=its + 5)
    lh, olh = data["loss_hist"], od["loss_hist"]
    assert float((lh - olh).abs().max()) <= 2e-7 * float(olh.abs().max())
    assert float((gp.raw_lengthscales.detach().cpu() - o.raw_lengthscales.detach()).abs().max()) <= 1e-10
    xt = torch.rand((npm, d), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt.to(DEV)).cpu()
    opm = o.post_mean(xt)
    assert float((pm - opm).abs().max()) <= 1e-7 * float(opm.abs().max())
    pv = gp.post_var(xt[:npv].to(DEV)).cpu()
    opv = o.post_var(xt[:npv])
    kxx = float(o.kernel(xt[:npv], xt[:npv]).detach().abs().max())
    assert float((pv - opv.detach()).abs().max()) <= 1e-8 * kxx


@pytest.mark.parametrize("m,d,alpha", [(16, 3, 2), (16, 5, 3), (17, 3, 2), (18, 2, 1), (19, 5, 2), (20, 5, 2),
                                         (20, 2, 2), (21, 3, 2), (22, 3, 2), (24, 1, 2)])
def test_half_length_fit_kernels_match_oracle(monkeypatch, m, d, alpha):
    """The lattice fit kernels for n >= 2^17 -- real-even (RE, regenerated parts; csrc/fgp_nll.hip
    k_*_re, the default), half-length (R2C, FGP_R2C=1; k_*_r2c) and full-length (FGP_R2C=0) -- on the
    same GP: eigenvalues (fgp_nll_lam) agree to 1e-12 relative; MLL and gradient of every variant
    against the CPU oracle (torch.fft + autograd, the reference's op sequence) to 2e-7 relative, the
    golden-fixture tolerance (tests/test_gpu_gp.py), with the nugget raised to 1e-3 (at the default
    1e-8 the MLL sums |y~|^2 / ev over eigenvalues at the nugget and every implementation's
    O(eps log n) eigenvalue error -- the reference's own included -- moves it by up to ~1e-5 relative at
    n = 2^21).  The R2C adjoint assumes dL/dlambda Hermitian; the kernel makes it exactly so (each
    mirror pair evaluated once, conjugated for the partner) -- without that, the rounding-level
    anti-Hermitian part, amplified by 1/ev^2 near the nugget, leaked 1e-5..1e-3 relative errors into
    the lengthscale gradient at n >= 2^19, d >= 3 (caught by this test).  The RE kernels treat lambda
    as exactly real and even (folded loss over n/2 + 1 frequencies, the gradient through the
    generated c_0 .. c_{n/2}); the oracle keeps the reference's complex arithmetic."""
    n = 2 ** m      # (n = 2^16: real-even and full-length kernels; FGP_R2C=1 runs the full-length ones there)
    ls = torch.linspace(0.6, 1.8, d)
    res = {}
    for mode in ("2", "1", "0"):
        monkeypatch.setenv("FGP_R2C", mode)
        gp = F.FastGPLattice(F.Lattice(d, seed=11), alpha=alpha, lengthscales=ls, noise=1e-3, device=DEV)
        x = gp.get_x_next(n)
        y = O.f_ackley(x.cpu())
        gp.add_y_next(y.to(DEV))
        with torch.no_grad():
            lam = gp.get_lam().clone()
        pb, G = gp._problem_batch()
        gen = gp._parts_gen(n) if mode == "2" else None
        assert mode != "2" or gen is not None
        eng = F.FusedMLL(gp._FAMILY, None if gen is not None else gp._k1parts(n), gp._ysq(pb, G),
                         gp.raw_scale.detach().reshape(-1),
                         gp.raw_lengthscales.detach().reshape(-1, gp.raw_lengthscales.shape[-1]),
                         gp.raw_noise.detach().reshape(-1), logdet_weight=1.0,
                         mll_const=F.fit_engine.mll_constant(1, n), gen=gen)
        loss, t1, t2, grad = eng.evaluate()
        res[mode] = (lam, float(loss), grad.detach().cpu().clone())
    o = O.OracleFastGP("lattice", x.cpu(), None, y, alpha=alpha, lengthscales=ls, noise=1e-3)
    oloss = o.mll_loss()[0]
    ogs, ogl = torch.autograd.grad(oloss, [o.raw_scale, o.raw_lengthscales])
    og = torch.cat([ogs.reshape(-1), ogl.reshape(-1)])
    (l1, f1, g1), (l0, f0, g0) = res["1"], res["0"]
    assert float((l1 - l0).abs().max()) <= 1e-12 * float(l0.abs().max())
    errs = {name: (abs(res[mode][1] - float(oloss)) / abs(float(oloss)),
                   float((res[mode][2][:1 + d] - og).abs().max()) / float(og.abs().max()))
            for name, mode in (("re", "2"), ("r2c", "1"), ("full", "0"))}
    assert all(e[0] <= 2e-7 and e[1] <= 2e-7 for e in errs.values()), errs
    # noise gradient (the third raw parameter block) against the full-length kernels
    assert abs(float(res["2"][2][-1] - g0[-1])) <= 2e-7 * float(g0.abs().max()), (res["2"][2], g0)


def test_even_generating_vector_entry_takes_r2c_and_matches_oracle():
    """The real-even kernels form a mirror pair's parts from one lattice index, which needs every z_j odd
    (M z_j = n/2 mod n); a generating vector with an even entry must take the R2C kernels (csrc/fgp_nll.hip
    to_nll) and still match the oracle (loss and gradient, 2e-7 relative, nugget 1e-3 as above)."""
    n, d = 2 ** 17, 2
    gp = F.FastGPLattice(F.Lattice(d, seed=5, generating_vector=[1, 182668]), lengthscales=torch.tensor([0.7, 1.3]),
                         noise=1e-3, device=DEV)
    x = gp.get_x_next(n)
    y = O.f_ackley(x.cpu())
    gp.add_y_next(y.to(DEV))
    pb, G = gp._problem_batch()
    gen = gp._parts_gen(n)
    assert gen is not None
    eng = F.FusedMLL(gp._FAMILY, None, gp._ysq(pb, G), gp.raw_scale.detach().reshape(-1),
                     gp.raw_lengthscales.detach().reshape(-1, gp.raw_lengthscales.shape[-1]),
                     gp.raw_noise.detach().reshape(-1), logdet_weight=1.0,
                     mll_const=F.fit_engine.mll_constant(1, n), gen=gen)
    assert eng.partials.numel() >= G * (4 + d) * ((n >> 13) + 1)   # R2C block count fits the workspace
    loss, _, _, grad = eng.evaluate()
    o = O.OracleFastGP("lattice", x.cpu(), None, y, lengthscales=torch.tensor([0.7, 1.3]), noise=1e-3)
    oloss = o.mll_loss()[0]
    ogs, ogl = torch.autograd.grad(oloss, [o.raw_scale, o.raw_lengthscales])
    og = torch.cat([ogs.reshape(-1), ogl.reshape(-1)])
    assert abs(loss - float(oloss)) <= 2e-7 * abs(float(oloss))
    assert float((grad.cpu()[:1 + d] - og).abs().max()) <= 2e-7 * float(og.abs().max())


@pytest.mark.parametrize("m,d,alpha", [(17, 3, 2), (18, 2, 1), (19, 5, 2), (20, 3, 3)])
def test_half_length_post_var_matches_full_length_and_oracle(monkeypatch, m, d, alpha):
    """Posterior variance through the half-length (R2C) quadratic-form kernels (csrc/fgp_predict.hip
    k_qf_rows_r2c / k_qf_cols_r2c, lattice n >= 2^17) -- single GP (materialised points) and GPBatch
    (regenerated points, delta formed from the lattice index) -- against the full-length kernels
    (FGP_R2C=0) to 1e-10 K(x,x) and against the CPU oracle (abstract_gp.py:381-416) to 1e-8 K(x,x)."""
    n = 2 ** m
    xt = torch.rand((5, d), generator=torch.Generator().manual_seed(23))
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("FGP_R2C", mode)
        gps = []
        for s in (31, 32):
            gp = F.FastGPLattice(F.Lattice(d, seed=s), alpha=alpha, lengthscales=torch.linspace(0.7, 1.4, d), device=DEV)
            gp.add_y_next(O.f_ackley(gp.get_x_next(n).cpu()).to(DEV))
            gps.append(gp)
        with torch.no_grad():
            single = gps[0].post_var(xt.to(DEV)).cpu()
        b = F.GPBatch(gps)
        batched = b.post_var(xt.to(DEV)).cpu()
        res[mode] = (single, batched)
    o = O.OracleFastGP("lattice", gps[0].get_x(n=n).cpu(), None, gps[0].y.cpu(), alpha=alpha,
                       lengthscales=torch.linspace(0.7, 1.4, d))
    opv = o.post_var(xt)
    kxx = float(o.kernel(xt, xt).detach().abs().max())
    (s1, b1), (s0, b0) = res["1"], res["0"]
    assert float((s1 - s0).abs().max()) <= 1e-10 * kxx
    assert float((b1 - b0).abs().max()) <= 1e-10 * kxx
    assert float((s1 - opv).abs().max()) <= 1e-8 * kxx
    assert float((b1[0] - opv).abs().max()) <= 1e-8 * kxx


@pytest.mark.parametrize("family", ["lattice", "net"])
def test_post_mean_chunk_sizes_agree(family):
    """fgp_post_mean with 32 .. 1024 training points per workgroup (ops.post_mean_chunk picks fewer for
    small problems, so that n = 2^16, N = 256 fills the chip): the same sum in a different order.  The sum
    cancels heavily (|coeffs| ~ |y| / noise, noise = 1e-8), so the orders agree to the posterior-mean
    tolerance (1e-7 relative; measured 5e-9), not to the rounding of one term; the automatic choice is
    what FastGP*.post_mean runs and it matches the oracle."""
    n, d = 2 ** 16, 3
    if family == "lattice":
        gp = F.FastGPLattice(F.Lattice(d, seed=3), device=DEV)
    else:
        gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=3), device=DEV)
    x = gp.get_x_next(n)
    y = O.f_ackley(x.cpu())
    gp.add_y_next(y.to(DEV))
    xt = torch.rand((256, d), generator=torch.Generator().manual_seed(5)).to(DEV)
    assert F.ops.post_mean_chunk(n, 256) == 64 and F.ops.post_mean_chunk(2 ** 20, 256) == 1024
    with torch.no_grad():
        coeffs = gp.coeffs.reshape(1, n)
        z = gp._points_T(n)
        hyp = gp._hyp_rows(gp._has_batch_params())
        outs = [F.ops.post_mean_matfree(gp._FAMILY, xt, z, hyp, coeffs, alphas=gp._alphas, tbits=gp._tbits(), chunk=c)
                for c in (1024, 256, 64, 32)]
        pm = gp.post_mean(xt)
    ref = outs[0]
    for o in outs[1:]:
        assert float((o - ref).abs().max()) <= 1e-7 * float(ref.abs().max())
    assert torch.equal(pm.reshape(-1), outs[2].reshape(-1))    # the automatic chunk (64) bit for bit
    o = O.OracleFastGP(family, x.cpu(), gp.get_xb().cpu() if family == "net" else None, y, alpha=gp._alphas[0],
                       t=getattr(gp, "t", None))
    opm = o.post_mean(xt.cpu())
    assert float((pm.cpu() - opm).abs().max()) <= 1e-7 * float(opm.abs().max())


@pytest.mark.parametrize("family", ["lattice", "net"])
def test_post_mean_output_blocks_in_one_launch_equal_block_launches(family):
    """fgp_post_mean with every output its own hyper-parameters and B > 4 (ABI 16: the blocks of 4 outputs as the
    problems of ONE launch, the remainder in a second) against one launch per block of <= 4 outputs at the same
    training chunk: the same arithmetic, bit for bit (B = 10: two full blocks and a block of 2)."""
    n, d, B = 2 ** 14, 3, 10
    if family == "lattice":
        gp = F.FastGPLattice(F.Lattice(d, seed=3), device=DEV)
    else:
        gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=3), device=DEV)
    gp.get_x_next(n)
    g = torch.Generator().manual_seed(9)
    xt = torch.rand((300, d), generator=g).to(DEV)
    z = gp._points_T(n)
    hyp = torch.cat([torch.rand((B, 1), generator=g) + 0.5, torch.rand((B, d), generator=g) + 0.3], 1).to(DEV)
    coeffs = torch.randn((B, n), generator=g).to(DEV)
    kw = dict(alphas=gp._alphas, tbits=gp._tbits(), chunk=512)
    one = F.ops.post_mean_matfree(gp._FAMILY, xt, z, hyp, coeffs, **kw)
    blocks = torch.cat([F.ops.post_mean_matfree(gp._FAMILY, xt, z, hyp[b:b + 4], coeffs[b:b + 4], **kw)
                        for b in range(0, B, 4)])
    assert one.shape == (B, 300)
    assert torch.equal(one, blocks)
