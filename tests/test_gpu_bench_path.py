"""Parity of the exact path bench.py times (BASELINE config C4, one GPU's share): a GPBatch of P = 8
randomly shifted lattice GPs (seeds 1000..1007, d = 5) through bench.step_batched -- by default the
spectral fit path (fit_engine.spectral_wanted: one set of part-product spectra shared by the 8 problems,
one fused k_spec_tile launch per Rprop iteration), the coefficient solve from the spectra
(fgp_spec_inv_eig + fgp_ifftbr_real_rf), fgp_post_mean_batched and fgp_post_var_batched with regenerated
training points; and, forced with FGP_FIT_PATH=transform, the real-even transform fit kernels the
spectral path replaced (still selected for d > 6 or n >= 2^22).

Per GP, against
  * the CPU oracle (oracle/fgp_oracle.py, the reference's op sequence: abstract_gp.py:152-416) at the
    golden-fixture tolerances: MLL trajectory 2e-7 relative, fitted raw lengthscales 1e-10,
    post_mean 1e-7 relative, post_var 1e-8 K(x,x) absolute;
  * the same GP fitted on its own (FastGPLattice.fit): loss history and fitted parameters bit for bit;
and the step is idempotent across bench's reset (a second step reproduces the first bit for bit).
"""
import argparse

import pytest
import torch

import bench
import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O
from tests.gpu_fixtures import DEV, abs_err, rel_err

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)

ITERS = 5


@pytest.mark.parametrize("m,path", [(17, "spectral"), (20, "spectral"), (20, "transform")])
def test_bench_step_matches_oracle_and_individual_fits(monkeypatch, m, path):
    if path == "transform":
        monkeypatch.setenv("FGP_FIT_PATH", "transform")
    monkeypatch.setenv("FGP_PARTS_GEN", "1")
    d, n, P = 5, 2 ** m, 8
    seeds = bench.shard_seeds(0, 1, P)
    assert seeds == list(range(1000, 1008))
    dev = torch.device(DEV, 0)
    sh = bench.Shifts(F, d, n, seeds, dev)
    assert sh.batch._source()[1] is not None, "the bench path regenerates the lattice parts"
    g = torch.Generator().manual_seed(17)
    xm = torch.rand((8, d), generator=g)
    xv = torch.rand((2, d), generator=g)
    args = argparse.Namespace(fit_iters=ITERS)
    data, pm, pv = bench.step_batched(sh, args, xm.to(dev), xv.to(dev), store_loss_hist=True)
    pm, pv = pm.cpu(), pv.cpu()
    raw = sh.batch.raw().cpu().clone()
    # idempotent across the bench's reset
    data2, pm2, pv2 = bench.step_batched(sh, args, xm.to(dev), xv.to(dev), store_loss_hist=True)
    for a, b in zip(data, data2):
        assert torch.equal(a["loss_hist"], b["loss_hist"])
    assert torch.equal(pm, pm2.cpu()) and torch.equal(pv, pv2.cpu())
    for p, seed in enumerate(seeds):
        gp_b = sh.gps[p]
        x = gp_b.get_x(n=n).cpu()
        y = sh.y[p].cpu()
        # individually fitted GP: bit for bit
        solo = F.FastGPLattice(F.Lattice(d, seed=seed, randomize="SHIFT"), device=DEV)
        xs = solo.get_x_next(n)
        assert torch.equal(xs.cpu(), x)
        solo.add_y_next(sh.y[p].clone())
        sd = solo.fit(iterations=ITERS, verbose=0, store_loss_hist=True, stop_crit_wait_iterations=ITERS + 1)
        assert sd["iterations"] == data[p]["iterations"] == ITERS
        assert torch.equal(sd["loss_hist"], data[p]["loss_hist"]), (p, sd["loss_hist"], data[p]["loss_hist"])
        assert torch.equal(solo.raw_lengthscales.detach().cpu().reshape(-1), raw[p, 1:1 + d])
        assert torch.equal(solo.raw_scale.detach().cpu().reshape(-1), raw[p, :1])
        with torch.no_grad():
            assert rel_err(pm[p], solo.post_mean(xm.to(DEV))) <= 1e-9
            kxx_s = float(solo._kdiag(xv.to(DEV)).abs().max())
            assert abs_err(pv[p], solo.post_var(xv.to(DEV))) <= 1e-10 * kxx_s
        # CPU oracle (the reference's op sequence)
        o = O.OracleFastGP("lattice", x, None, y, alpha=2)
        od = o.fit(iterations=ITERS, stop_crit_wait_iterations=ITERS + 1)
        lh, olh = data[p]["loss_hist"], od["loss_hist"]
        assert float((lh - olh).abs().max()) <= 2e-7 * float(olh.abs().max()), (p, lh, olh)
        assert float((raw[p, 1:1 + d] - o.raw_lengthscales.detach().reshape(-1)).abs().max()) <= 1e-10
        opm = o.post_mean(xm)
        assert float((pm[p] - opm).abs().max()) <= 1e-7 * float(opm.abs().max())
        opv = o.post_var(xv)
        kxx = float(o.kernel(xv, xv).detach().abs().max())
        assert float((pv[p] - opv).abs().max()) <= 1e-8 * kxx


def test_fused_iteration_handoff_is_consistent(monkeypatch):
    """The relaxed last-arriver hand-off of k_spec_tile (sc1 partial stores, vmcnt(0), a relaxed agent-scope
    add: MI355X_MICROARCH.md hand-off row 1) checked in the suite, once: fgp_handoff_check arms a per-group
    XOR of the partials' bits accumulated by the storing waves before their arrival, and every group's last
    arriver recomputes it from what it reads -- C4's 16 groups x 40 iterations, no mismatch allowed."""
    import ctypes
    from fastgaussianprocesses_amd import _native as N
    monkeypatch.setenv("FGP_PARTS_GEN", "1")
    d, n, P, iters = 5, 2 ** 20, 8, 40
    dev = torch.device(DEV, 0)
    sh = bench.Shifts(F, d, n, bench.shard_seeds(0, 1, P), dev)
    g = torch.Generator().manual_seed(17)
    xm, xv = torch.rand((8, d), generator=g).to(dev), torch.rand((2, d), generator=g).to(dev)
    out = (ctypes.c_ulonglong * 2)()
    N.call("fgp_handoff_check", 1, out)
    try:
        data, _, _ = bench.step_batched(sh, argparse.Namespace(fit_iters=iters), xm, xv, store_loss_hist=True)
    finally:
        N.call("fgp_handoff_check", 0, out)
    assert all(dd["iterations"] == iters for dd in data)
    groups = 512 // 32                      # nb = 512 k blocks at n = 2^20, kSpecGroup = 32
    # one k_spec_tile launch per evaluated iteration (iterations 0 .. iters: the last evaluates only)
    assert out[0] % groups == 0 and iters * groups <= out[0] <= (iters + 1) * groups, (out[0], out[1])
    assert out[1] == 0, "last arrivers read %d partial groups that differ from what was stored" % out[1]
