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


def test_bench_gpus_2_runs_two_ranks(tmp_path):
    """`bench.py --gpus 2` without a launcher starts two ranks itself (torch.distributed.run as a child process,
    before any GPU call in the parent) -- here both ranks on cuda:0 over gloo (FGP_BENCH_DEVICE /
    FGP_BENCH_BACKEND) -- and relays rank 0's line: n_gpus 2, 4 global shifts, the CPU baseline present; each
    rank's fitted parameters and predictions equal those of an N = 1 run over the same four seeds bit for bit
    (rank r owns seeds 1000 + 2r, 1001 + 2r: bench.shard_seeds)."""
    import json
    import os
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--log2n", "14", "--steps", "1", "--warmup", "1", "--no-secondary", "--no-paper", "--no-multitask",
              "--fit-iters", "10", "--n-mean", "8", "--n-var", "2"]
    env = dict(os.environ, FGP_BENCH_DEVICE="0", FGP_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    runs = {}
    for gpus, shifts in ((2, 2), (1, 4)):
        out = tmp_path / ("n%d" % gpus)
        cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--shifts", str(shifts),
               "--dump", str(out)] + common
        r = subprocess.run(cmd, cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=100)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        runs[gpus] = (json.loads(lines[0]), out)
    line2, out2 = runs[2]
    assert line2["n_gpus"] == 2 and line2["config"]["global_shifts"] == 4
    assert line2["cpu_baseline"] is not None and line2["cpu_baseline"]["value"] > 0
    one = np.load(runs[1][1] / "rank0.npz")
    assert list(one["seeds"]) == [1000, 1001, 1002, 1003]
    for r in range(2):
        got = np.load(out2 / ("rank%d.npz" % r))
        assert list(got["seeds"]) == [1000 + 2 * r, 1001 + 2 * r]
        for k in ("raw", "post_mean", "post_var"):
            assert np.array_equal(got[k], one[k][2 * r:2 * r + 2]), (r, k)


# The exact benched C4 work (n = 2^20, d = 5, alpha = 2, nugget 1e-8, 50 Rprop iterations with early stopping off,
# post_mean, post_var) against the REAL reference (tests/golden/make_golden_c4.py -> c4_m20_d5_it50.npz, shift seeds
# 1000 and 1001).  Tolerances = 5x the reference's own torch.fft vs numpy-pocketfft spread over the same 50
# iterations (profiles/r05_c4_backend_spread.json: loss history 7.1e-9 of its largest value, post_mean 2.2e-9
# relative, post_var 6e-16 K(x, x), fitted parameters identical); the variance keeps the golden tests' 1e-8 K(x, x)
# and the parameters their 1e-10.
C4_TOL = dict(loss=3.6e-8, pmean=1.1e-8, pvar_kxx=1e-8, params=1e-10)


def test_bench_step_50_iterations_matches_reference(monkeypatch):
    """bench.step_batched exactly as timed (P = 8 shifts, 50 iterations, the spectral fused fit, the coefficients
    from the spectra, batched post_mean / post_var) for the fixture's two shifts against the reference's
    trajectories and posteriors -- the sign-driven Rprop trajectory pinned over the whole benched length."""
    import os
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c4_m20_d5_it50.npz"))
    d, n, its = int(g["d"]), 2 ** int(g["m"]), int(g["its"])
    seeds = bench.shard_seeds(0, 1, 8)
    assert list(g["seeds"]) == seeds[:2]
    dev = torch.device(DEV, 0)
    sh = bench.Shifts(F, d, n, seeds, dev)
    xt = torch.from_numpy(g["x_test"])
    args = argparse.Namespace(fit_iters=its)
    data, pm, pv = bench.step_batched(sh, args, xt.to(dev), xt[:2].to(dev), store_loss_hist=True)
    pm, pv = pm.cpu().numpy(), pv.cpu().numpy()
    raw = sh.batch.raw().cpu().numpy()
    for p in range(2):
        gp = sh.gps[p]
        assert np.array_equal(gp.seq.z[:d], g["z"]) and np.array_equal(gp.seq.shift, g["shift"][p])
        assert data[p]["iterations"] == its
        lh, ref = data[p]["loss_hist"].numpy(), g["loss_hist"][p]
        assert lh.shape == ref.shape
        assert np.abs(lh - ref).max() <= C4_TOL["loss"] * np.abs(ref).max(), (p, np.abs(lh - ref).max())
        assert np.abs(raw[p, :1] - g["raw_scale"][p]).max() <= C4_TOL["params"]
        assert np.abs(raw[p, 1:1 + d] - g["raw_lengthscales"][p]).max() <= C4_TOL["params"]
        assert np.abs(pm[p] - g["pmean"][p]).max() <= C4_TOL["pmean"] * np.abs(g["pmean"][p]).max()
        assert (np.abs(pv[p] - g["pvar"][p]) <= C4_TOL["pvar_kxx"] * g["kxx"][p]).all()


# The benched C2 / C3 work (bench.SingleGP: n = 2^16, d = 3, alpha = 2, default nugget; 50 Rprop iterations with early
# stopping off, post_mean, post_var) against the REAL reference (tests/golden/make_golden_c23.py -> c2_m16_d3_it50.npz,
# c3_m16_d3_a2_it50.npz).  Tolerances = 5x the reference's own spread between two correct transforms over the same 50
# iterations (profiles/r06_c23_backend_spread.json: C2 torch.fft vs pocketfft -- loss history 6.2e-8 of its largest
# value, post_mean 2.6e-9, post_var 5.4e-16 K(x, x), parameters identical; C3 two FWHT butterfly orders -- loss 2.4e-14,
# post_mean 1.4e-13, post_var 1.2e-15 K(x, x), parameters identical), with the floors of the golden tests where 5x the
# spread is below them: fitted parameters 1e-10, post_var 1e-8 K(x, x); and for C3, whose MLL the two FWHTs round
# identically to 2e-14, the loss / post_mean floors C23_FLOOR (the spectral fit sums lambda = scale sum_S l^S Phi_S in
# another order than ft(k1): a rounding-level difference the reference's two transforms do not show).
C23_TOL = {"c2_m16_d3_it50": dict(loss=3.1e-7, pmean=1.3e-8, pvar_kxx=1e-8, params=1e-10),
           "c3_m16_d3_a2_it50": dict(loss=1.2e-13, pmean=7.2e-13, pvar_kxx=1e-8, params=1e-10)}
C23_FLOOR = dict(loss=1e-11, pmean=1e-10)


@pytest.mark.parametrize("name", sorted(C23_TOL))
def test_bench_c2_c3_50_iterations_match_reference(name):
    """bench.step_single exactly as timed for C2 (FastGPLattice) and C3 (FastGPDigitalNetB2, alpha = 2): fitted
    parameters, post_mean at the fixture's 16 points and post_var at its first 2 against the reference after 50
    iterations; the loss history of the same fit (store_loss_hist) against the reference's."""
    import os
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"))
    family, m, d, its = str(g["family"]), int(g["m"]), int(g["d"]), int(g["its"])
    dev = torch.device(DEV, 0)
    sg = bench.SingleGP(F, family, m, d, dev)
    seq = sg.gp.seq if hasattr(sg.gp, "seq") else sg.gp.seqs[0]
    if family == "lattice":
        assert np.array_equal(np.asarray(seq.z)[:d], g["z"]) and np.array_equal(seq.shift, g["shift"])
    else:
        assert np.array_equal(np.asarray(seq.C, dtype=np.uint64)[:d, :g["C"].shape[1]], g["C"].astype(np.uint64))
        assert np.array_equal(np.asarray(seq.shift, dtype=np.uint64), g["shift"].astype(np.uint64))
    xt = torch.from_numpy(g["x_test"])
    args = argparse.Namespace(fit_iters=its)
    pm, pv = bench.step_single(sg, args, xt.to(dev), xt[:2].to(dev))
    pm, pv = pm.cpu().numpy(), pv.cpu().numpy()
    rs, rl = (sg.gp.raw_scale.detach().cpu().numpy().reshape(-1), sg.gp.raw_lengthscales.detach().cpu().numpy().reshape(-1))
    sg.reset()
    data = sg.gp.fit(iterations=its, stop_crit_wait_iterations=its + 1, verbose=0, store_loss_hist=True)
    tol = C23_TOL[name]
    lh, ref = data["loss_hist"].numpy(), g["loss_hist"]
    assert data["iterations"] == its and lh.shape == ref.shape
    e_loss = np.abs(lh - ref).max() / np.abs(ref).max()
    e_pm = np.abs(pm - g["pmean"]).max() / np.abs(g["pmean"]).max()
    errs = dict(loss=e_loss, pmean=e_pm, scale=np.abs(rs - g["raw_scale"]).max(),
                lengthscales=np.abs(rl - g["raw_lengthscales"]).max(),
                pvar_kxx=(np.abs(pv - g["pvar"]) / np.abs(g["kxx"])).max())
    assert e_loss <= max(tol["loss"], C23_FLOOR["loss"]), errs
    assert errs["scale"] <= tol["params"] and errs["lengthscales"] <= tol["params"], errs
    assert e_pm <= max(tol["pmean"], C23_FLOOR["pmean"]), errs
    assert errs["pvar_kxx"] <= tol["pvar_kxx"], errs
