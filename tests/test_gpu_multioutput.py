"""BASELINE config C5 (multi-output FastGPLattice, n = 2^18) on the GPU, fp64:

* shared hyper-parameters (the reference's default shape_scale = [1], shape_lengthscales = [d]):
  the fused fit over Y = sum_b |y~_b|^2 (one eigen-problem) and the GEMM-shaped posterior mean of many
  outputs (fgp_kernel_rows + library GEMM, ops.post_mean_gemm);
* per-output hyper-parameters (docs/examples/batch_multitask/fgp_lattice.ipynb cell 6:
  shape_scale = [B, 1], shape_lengthscales = [B, d]): B eigen-problems, one summed loss;
* distributed.fit_sharded across two processes (gloo, both ranks on cuda:0): each rank transforms its
  own outputs, one all-reduce of Y, identical device fits -- equal to the unsharded fit.
Against the CPU oracle (the reference's op sequence, abstract_gp.py:152-416 with shape_batch) at the
golden-fixture tolerances (tests/test_gpu_gp.py).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O
from tests.gpu_fixtures import DEV, rel_err

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)


def _data(x, B):
    f = O.f_ackley(x)
    g = torch.Generator().manual_seed(5)
    return torch.stack([f * (1 + b / B) + 0.01 * torch.randn(f.shape, generator=g) for b in range(B)])


def _c5_data(x, B, seed=5):
    """bench.py's / tests/golden/make_golden_c5.py's C5 observations: f_ackley(x) (1 + b / B) + 0.01 randn."""
    g = torch.Generator().manual_seed(seed)
    noise = torch.randn((B, x.shape[0]), generator=g, dtype=torch.float64)
    b = torch.arange(B, dtype=torch.float64)[:, None]
    return O.f_ackley(x)[None, :] * (1 + b / B) + 0.01 * noise


# Tolerances of the benched C5 regime (2^18 x 512 outputs, nugget 1e-8) = 5x the REAL reference's own
# spread between its torch.fft and numpy-pocketfft backends at that configuration
# (tests/golden/make_golden_c5.py -> profiles/r03_c5_backend_spread.json: loss history 4.9e-7 relative,
# post_mean 1.08e-7 relative, post_var 1e-15 K(x,x), fitted parameters identical).
C5_TOL = dict(loss=2.5e-6, pmean=5.4e-7, pvar_kxx=1e-8, params=1e-10)


@pytest.mark.parametrize("mixed", [False, True])
def test_benched_c5_regime_matches_reference(mixed):
    """The C5 configuration bench.py times: n = 2^18, d = 3, 512 outputs sharing the default hyper-parameters,
    the default nugget 1e-8, fit(iterations=3) (early stopping off), post_mean at 16 and post_var at 2 test
    points -- against the REAL reference's results on the same points and data (tests/golden/
    c5_m18_d3_b512*.npz).  mixed: float32 observations (widened exactly into the fp64 half-spectrum transform
    that feeds Y and the coefficients, ABI 16) against the reference on the same float32-rounded data; its loss
    tolerance keeps the 1e-6 allowance of the earlier complex64 Y (now fp64: the allowance is unused)."""
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(__file__), "golden",
                             "c5_m18_d3_b512%s.npz" % ("_f32data" if mixed else "")))
    m, d, B, its = int(g["m"]), int(g["d"]), int(g["B"]), int(g["its"])
    seq = F.Lattice(d, randomize="SHIFT", generating_vector=g["z"], shift=g["shift"])
    gp = F.FastGPLattice(seq, alpha=2, shape_batch=[B], device=DEV,
                         data_dtype=torch.float32 if mixed else torch.float64)
    x = gp.get_x_next(2 ** m).cpu()
    y = _c5_data(x, B)
    gp.add_y_next((y.float() if mixed else y).to(DEV))
    data = gp.fit(iterations=its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=its + 5)
    lh = data["loss_hist"]
    olh = torch.from_numpy(g["loss_hist"])
    assert rel_err(lh, olh) <= C5_TOL["loss"] + (1e-6 if mixed else 0.0)
    assert float((gp.raw_lengthscales.detach().cpu() - torch.from_numpy(g["raw_lengthscales"])).abs().max()) <= C5_TOL["params"]
    assert float((gp.raw_scale.detach().cpu() - torch.from_numpy(g["raw_scale"])).abs().max()) <= C5_TOL["params"]
    xt = torch.from_numpy(g["x_test"])
    pm = gp.post_mean(xt.to(DEV)).cpu()
    assert pm.shape == tuple(g["pmean"].shape)
    assert rel_err(pm, g["pmean"]) <= C5_TOL["pmean"]
    pv = gp.post_var(xt[:g["pvar"].shape[-1]].to(DEV)).cpu()
    assert float((pv - torch.from_numpy(g["pvar"])).abs().max()) <= C5_TOL["pvar_kxx"] * float(g["kxx"])


# The per-output regime bench.py also times (C5 per-output: shape_scale = [512, 1], shape_lengthscales = [512, 3],
# nugget 1e-8): 5x the REAL reference's torch.fft vs numpy-pocketfft spread there (tests/golden/
# make_golden_c5.py --per-output -> profiles/r04_c5_po_backend_spread.json: loss history 7.1e-7 relative,
# post_mean 1.7e-7 relative, post_var 2.8e-16 of each output's K(x, x), fitted parameters identical); the
# variance keeps the 1e-8 K(x, x) of the golden tests.
C5_PO_TOL = dict(loss=3.6e-6, pmean=8.3e-7, pvar_kxx=1e-8, params=1e-10)


def test_benched_c5_per_output_regime_matches_reference():
    """C5 per-output as bench.py times it: 512 eigen-problems on one point set (the sliced k_spec_tile<3, 4>,
    the parallel many-problem step k_spec_step_many, fgp_spec_post_var at G = 512), fit(iterations=3),
    post_mean at 16 and post_var at 2 test points -- against the REAL reference (tests/golden/
    c5_m18_d3_b512_po.npz; the reference ran in chunks of 64 outputs, its per-output problems being
    independent)."""
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c5_m18_d3_b512_po.npz"))
    m, d, B, its = int(g["m"]), int(g["d"]), int(g["B"]), int(g["its"])
    seq = F.Lattice(d, randomize="SHIFT", generating_vector=g["z"], shift=g["shift"])
    gp = F.FastGPLattice(seq, alpha=2, shape_batch=[B], shape_scale=[B, 1], shape_lengthscales=[B, d], device=DEV)
    x = gp.get_x_next(2 ** m).cpu()
    gp.add_y_next(_c5_data(x, B).to(DEV))
    data = gp.fit(iterations=its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=its + 5)
    assert rel_err(data["loss_hist"], torch.from_numpy(g["loss_hist"])) <= C5_PO_TOL["loss"]
    for k in ("raw_lengthscales", "raw_scale"):
        assert float((getattr(gp, k).detach().cpu() - torch.from_numpy(g[k])).abs().max()) <= C5_PO_TOL["params"], k
    xt = torch.from_numpy(g["x_test"])
    pm = gp.post_mean(xt.to(DEV)).cpu()
    assert pm.shape == tuple(g["pmean"].shape)
    assert rel_err(pm, g["pmean"]) <= C5_PO_TOL["pmean"]
    pv = gp.post_var(xt[:g["pvar"].shape[-1]].to(DEV)).cpu()
    assert pv.shape == tuple(g["pvar"].shape)
    kxx = torch.from_numpy(np.abs(g["kxx_all"]))
    assert float(((pv - torch.from_numpy(g["pvar"])).abs() / kxx).max()) <= C5_PO_TOL["pvar_kxx"]


@pytest.mark.parametrize("per_output", [False, True])
def test_multi_output_fit_and_predict_match_oracle(per_output):
    m, d, B, its = 18, 3, 16, 3
    n = 2 ** m
    # nugget 1e-3: with 0.01 randn in the data the MLL at the default 1e-8 sums |y~|^2 / ev over
    # eigenvalues at the nugget, where every implementation's O(eps sqrt(n) lambda_max) eigenvalue
    # error (the reference's own FFT's included) is ~1e-5 relative (measured 1.6e-6 on the loss here;
    # tests/test_gpu_configs.py::test_half_length_fit_kernels_match_oracle raises it the same way)
    kw = dict(shape_batch=[B], noise=1e-3)
    okw = dict(noise=1e-3)
    if per_output:
        kw.update(shape_scale=[B, 1], shape_lengthscales=[B, d])
        okw.update(shape_scale=(B, 1), shape_lengthscales=(B, d))
    gp = F.FastGPLattice(F.Lattice(d, seed=7), device=DEV, **kw)
    x = gp.get_x_next(n).cpu()
    y = _data(x, B)
    gp.add_y_next(y.to(DEV))
    data = gp.fit(iterations=its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=its + 5)
    o = O.OracleFastGP("lattice", x, None, y, alpha=2, **okw)
    od = o.fit(iterations=its, stop_crit_wait_iterations=its + 5)
    lh, olh = data["loss_hist"], od["loss_hist"]
    assert float((lh - olh).abs().max()) <= 2e-7 * float(olh.abs().max())
    assert float((gp.raw_lengthscales.detach().cpu() - o.raw_lengthscales.detach()).abs().max()) <= 1e-10
    xt = torch.rand((24, d), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt.to(DEV)).cpu()
    opm = o.post_mean(xt)
    assert pm.shape == opm.shape == (B, 24)
    assert rel_err(pm, opm) <= 1e-7
    pv = gp.post_var(xt[:4].to(DEV)).cpu()
    opv = o.post_var(xt[:4])
    kxx = float(o.kernel(xt[:4], xt[:4]).detach().abs().max())
    assert pv.shape == opv.shape
    assert float((pv - opv).abs().max()) <= 1e-8 * kxx


def test_mixed_precision_multi_output_matches_oracle():
    """data_dtype=float32 (the fp32 C5 path): fp32 observations stored, widened exactly on load into ONE fp64
    Hermitian-half transform (fgp_fftbr_real_half_f32, ABI 16) that feeds the MLL's Y and the coefficients; fp64
    eigenvalues / fit / posteriors; get_ytilde keeps the API's complex64 ft(y).  Against the fp64 oracle on the same
    fp32-rounded observations: loss trajectory 2e-6 relative, fitted lengthscales 1e-10, posterior mean 1e-7,
    posterior variance 1e-8 K(x,x)."""
    m, d, B, its = 18, 3, 16, 4
    n = 2 ** m
    gp = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[B], noise=1e-3, device=DEV, data_dtype=torch.float32)
    x = gp.get_x_next(n).cpu()
    y32 = _data(x, B).float()
    gp.add_y_next(y32.to(DEV))
    assert gp.y.dtype == torch.float32 and gp.get_ytilde(0).dtype == torch.complex64
    data = gp.fit(iterations=its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=its + 5)
    o = O.OracleFastGP("lattice", x, None, y32.double(), alpha=2, noise=1e-3)
    od = o.fit(iterations=its, stop_crit_wait_iterations=its + 5)
    lh, olh = data["loss_hist"], od["loss_hist"]
    assert float((lh - olh).abs().max()) <= 2e-6 * float(olh.abs().max())
    assert float((gp.raw_lengthscales.detach().cpu() - o.raw_lengthscales.detach()).abs().max()) <= 1e-10
    xt = torch.rand((24, d), generator=torch.Generator().manual_seed(17))
    assert rel_err(gp.post_mean(xt.to(DEV)), o.post_mean(xt)) <= 1e-7
    kxx = float(o.kernel(xt[:4], xt[:4]).detach().abs().max())
    assert float((gp.post_var(xt[:4].to(DEV)).cpu() - o.post_var(xt[:4])).abs().max()) <= 1e-8 * kxx


def test_gemm_posterior_mean_equals_matrix_free():
    """ops.post_mean_gemm (kernel rows + library GEMM) against the matrix-free HIP contraction
    (fgp_post_mean, 4 outputs per launch) on the same coefficients."""
    from fastgaussianprocesses_amd import ops
    m, d, B = 16, 4, 12
    gp = F.FastGPLattice(F.Lattice(d, seed=3), device=DEV)
    gp.get_x_next(2 ** m)
    z = gp._points_T(2 ** m)
    hyp = torch.tensor([[1.3, 0.7, 1.1, 0.9, 1.6]], device=DEV)
    c = torch.randn((B, 2 ** m), generator=torch.Generator().manual_seed(2)).to(DEV)
    xt = torch.rand((300, d), generator=torch.Generator().manual_seed(4)).to(DEV)
    g = ops.post_mean_gemm(ops.LATTICE, xt, z, hyp, c, alphas=[2] * d)
    ref = torch.cat([ops.post_mean_matfree(ops.LATTICE, xt, z, hyp, c[b0:b0 + 4], alphas=[2] * d)
                     for b0 in range(0, B, 4)])
    assert rel_err(g, ref) <= 1e-12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, B, m, d, its, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.set_default_dtype(torch.float64)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fastgaussianprocesses_amd.distributed import fit_sharded, output_shard
        n = 2 ** m
        a, b = output_shard(B, rank, world)
        gp = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[b - a], device="cuda:0")
        x = gp.get_x_next(n).cpu()
        gp.add_y_next(_c5_data(x, B)[a:b].to("cuda:0"))
        data = fit_sharded(gp, B, iterations=its, store_loss_hist=True, stop_crit_wait_iterations=10)
        # (numpy by value: a tensor would travel as a shared file descriptor, lost if the worker exits first)
        q.put((rank, data["iterations"], data["loss_hist"].numpy().copy(), gp.raw_lengthscales.detach().cpu().numpy().copy(),
               gp.raw_scale.detach().cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B,m,its", [(10, 16, 6), (512, 18, 3)])
def test_fit_sharded_two_processes_equals_unsharded(B, m, its):
    """distributed.fit_sharded over two processes (gloo, both on cuda:0), outputs split B/2 + B/2 -- also
    at the benched C5 size (2^18 x 512: 256 + 256) -- equals the unsharded fit on one process."""
    d, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, B, m, d, its, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[B], device=DEV)
    x = full.get_x_next(2 ** m).cpu()
    full.add_y_next(_c5_data(x, B).to(DEV))
    ref = full.fit(iterations=its, verbose=0, store_loss_hist=True, stop_crit_wait_iterations=10)
    for _, its, lh, ls, sc in res:
        lh, ls, sc = torch.from_numpy(lh), torch.from_numpy(ls), torch.from_numpy(sc)
        assert its == ref["iterations"]
        assert rel_err(lh, ref["loss_hist"]) < 1e-10           # Y summed in another order
        assert rel_err(ls, full.raw_lengthscales) < 1e-10
    assert np.array_equal(res[0][3], res[1][3]) and np.array_equal(res[0][4], res[1][4])   # identical on every rank


def test_fp32_data_coefficients_same_with_and_without_graph():
    """data_dtype=float32: the coefficients come from an fp64 transform of the observations in grad mode
    too (it ran the fp32 transform there, O(1) relative error), so both modes agree to the
    coefficient tolerance of test_gpu_gp.py (1e-6: K^-1 y at cond(K) ~ n / noise; the two modes form
    lambda by different kernels, autograd ft(k1) vs the fused path)."""
    d, n = 2, 2 ** 12
    gp = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[3], device=DEV, data_dtype=torch.float32)
    x = gp.get_x_next(n)
    y = torch.stack([O.f_ackley(x.cpu()) * (1 + b) for b in range(3)]).to(DEV).float()
    gp.add_y_next(y)
    with torch.no_grad():
        c0 = gp.coeffs.clone()
    gp._cache = {}
    c1 = gp.coeffs.detach()
    assert rel_err(c1, c0) <= 1e-6


def _bench_secondary_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import argparse
    import torch.distributed as dist
    torch.set_default_dtype(torch.float64)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        args = argparse.Namespace(fit_iters=50, n_mean=64, n_var=4, c5_outputs=512, steps=1)
        got = {}
        lines = bench.secondary_configs(F, args, "cuda:0", rank, world, collect=got)
        q.put((rank, lines, got))
    finally:
        dist.destroy_process_group()


def test_bench_secondary_c5_lines_two_ranks_equal_one_rank():
    """bench.py's N > 1 C5 path, executed: bench.secondary_configs itself at world size 2 (gloo, both ranks on
    cuda:0) -- C5 with the outputs sharded over the ranks (distributed.fit_sharded: one Y all-reduce) and C5
    per-output (replicas of 256 outputs) -- against the same function at world size 1: every rank's fitted
    parameters equal the N = 1 fit's to 1e-10 (Y summed in another order; the per-output problems are
    independent), and its post_mean / post_var are the N = 1 run's rows of the outputs it owns."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_secondary_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import argparse
    import bench
    args = argparse.Namespace(fit_iters=50, n_mean=64, n_var=4, c5_outputs=512, steps=1)
    ref = {}
    bench.secondary_configs(F, args, DEV, 0, 1, collect=ref)
    for rank, lines, got in res:
        assert [ln["n_gpus"] for ln in lines] == [2, 2]
        assert all(ln["value"] > 0 for ln in lines)
        for case in ("C5", "C5 per-output"):
            r, o = ref[case], got[case]
            a, b = o["outputs"]
            assert (a, b) == bench.c5_shard(512, rank, world)
            for k in ("raw_scale", "raw_lengthscales"):
                rv = r[k][a:b] if (case == "C5 per-output" and r[k].shape[0] == 512) else r[k]
                assert float((o[k] - rv).abs().max()) <= 1e-10, (case, k)
            assert rel_err(o["post_mean"], r["post_mean"][a:b]) <= 1e-9, case
            # (shared hyper-parameters: one posterior variance per test point for every output)
            pr = r["post_var"]
            pv_ref = pr[a:b] if (pr.dim() > 1 and pr.shape[0] == 512) else pr
            assert o["post_var"].shape == pv_ref.shape, case
            kxx = float(pr.abs().max()) + 1e-300
            assert float((o["post_var"] - pv_ref).abs().max()) <= 1e-9 * max(kxx, 1.0), case


# The benched C5 work at its benched length (bench.MultiOutputGP: n = 2^18, d = 3, 512 outputs, shared hyper-parameters,
# nugget 1e-8; bench.step_single: fit 50 Rprop iterations with early stopping off, post_mean, post_var) against the REAL
# reference (tests/golden/make_golden_c5.py --its 50 -> c5_m18_d3_b512[_f32data]_it50.npz).  Tolerances = 5x the
# reference's own torch.fft vs numpy-pocketfft spread over the same 50 iterations (profiles/r06_c5_backend_spread.json:
# loss history 4.9e-7 relative, post_mean 1.7e-7 relative, post_var 1e-15 K(x,x), fitted parameters identical), with
# the golden tests' floors: parameters 1e-10, post_var 1e-8 K(x,x).
C5_50_TOL = dict(loss=2.5e-6, pmean=8.4e-7, pvar_kxx=1e-8, params=1e-10)


@pytest.mark.parametrize("mixed", [False, True])
def test_bench_c5_50_iterations_matches_reference(mixed):
    """bench.step_single exactly as timed for the C5 line (mixed: the fp32-observation line) at the fixture's test
    points: fitted parameters, post_mean (16 points), post_var (2 points); the loss history of the same 50-iteration
    fit (store_loss_hist) -- the sign-driven Rprop trajectory pinned over the whole benched length."""
    import argparse
    import numpy as np
    import bench
    g = np.load(os.path.join(os.path.dirname(__file__), "golden",
                             "c5_m18_d3_b512%s_it50.npz" % ("_f32data" if mixed else "")))
    m, d, B, its = int(g["m"]), int(g["d"]), int(g["B"]), int(g["its"])
    dev = torch.device(DEV, 0)
    sg = bench.MultiOutputGP(F, m, d, B, dev, data_dtype=torch.float32 if mixed else torch.float64)
    assert np.array_equal(np.asarray(sg.gp.seq.z)[:d], g["z"]) and np.array_equal(sg.gp.seq.shift, g["shift"])
    xt = torch.from_numpy(g["x_test"])
    pm, pv = bench.step_single(sg, argparse.Namespace(fit_iters=its), xt.to(dev), xt[:g["pvar"].shape[-1]].to(dev))
    rs, rl = sg.gp.raw_scale.detach().cpu(), sg.gp.raw_lengthscales.detach().cpu()
    sg.reset()
    data = sg.gp.fit(iterations=its, stop_crit_wait_iterations=its + 1, verbose=0, store_loss_hist=True)
    assert data["iterations"] == its
    errs = dict(loss=rel_err(data["loss_hist"], g["loss_hist"]),
                scale=float((rs - torch.from_numpy(g["raw_scale"])).abs().max()),
                lengthscales=float((rl - torch.from_numpy(g["raw_lengthscales"])).abs().max()),
                pmean=rel_err(pm, g["pmean"]),
                pvar_kxx=float((pv.cpu() - torch.from_numpy(g["pvar"])).abs().max()) / float(g["kxx"]))
    assert pm.shape == tuple(g["pmean"].shape)
    assert errs["loss"] <= C5_50_TOL["loss"], errs
    assert errs["scale"] <= C5_50_TOL["params"] and errs["lengthscales"] <= C5_50_TOL["params"], errs
    assert errs["pmean"] <= C5_50_TOL["pmean"], errs
    assert errs["pvar_kxx"] <= C5_50_TOL["pvar_kxx"], errs


def test_bench_c5_per_output_50_iterations_matches_reference():
    """The C5 per-output line (512 independent eigen-problems on one point set) exactly as bench.step_single times it,
    50 iterations, against the REAL reference (tests/golden/make_golden_c5.py --per-output --its 50).  Over 50 sign-driven
    Rprop steps the reference's own torch.fft and pocketfft runs fork on ONE output (profiles/r06_c5_po_backend_spread.json:
    output 111; the other 511 end with identical parameters), so each output is held to the reference run it follows:
    parameters 1e-10 of the torch.fft run, or -- on a forked output only -- of the pocketfft run
    (c5_m18_d3_b512_po_it50_alt.npz); posterior means 5x the spread of the unforked outputs (2.6e-7 relative -> 1.3e-6)
    against the run the output follows; variances 1e-8 K(x,x); the summed loss history 5x the spread (7.1e-7 -> 3.6e-6)."""
    import argparse
    import json
    import numpy as np
    import bench
    here = os.path.dirname(__file__)
    g = np.load(os.path.join(here, "golden", "c5_m18_d3_b512_po_it50.npz"))
    alt = np.load(os.path.join(here, "golden", "c5_m18_d3_b512_po_it50_alt.npz"))
    forked = set(json.load(open(os.path.join(here, "..", "profiles", "r06_c5_po_backend_spread.json")))["outputs_forked"])
    m, d, B, its = int(g["m"]), int(g["d"]), int(g["B"]), int(g["its"])
    dev = torch.device(DEV, 0)
    sg = bench.MultiOutputGP(F, m, d, B, dev, per_output=True)
    xt = torch.from_numpy(g["x_test"])
    pm, pv = bench.step_single(sg, argparse.Namespace(fit_iters=its), xt.to(dev), xt[:g["pvar"].shape[-1]].to(dev))
    pm, pv = pm.cpu().numpy(), pv.cpu().numpy()
    rs = sg.gp.raw_scale.detach().cpu().numpy().reshape(B, -1)
    rl = sg.gp.raw_lengthscales.detach().cpu().numpy().reshape(B, -1)
    sg.reset()
    data = sg.gp.fit(iterations=its, stop_crit_wait_iterations=its + 1, verbose=0, store_loss_hist=True)
    assert rel_err(data["loss_hist"], g["loss_hist"]) <= 3.6e-6
    kxx = np.abs(g["kxx_all"])
    follows = {}
    for b in range(B):
        errs = []
        for name, run in (("torch", g), ("pocketfft", alt)):
            errs.append(max(np.abs(rs[b] - run["raw_scale"].reshape(B, -1)[b]).max(),
                            np.abs(rl[b] - run["raw_lengthscales"].reshape(B, -1)[b]).max()))
        if errs[0] <= 1e-10:
            follows[b] = g
        else:
            assert b in forked and errs[1] <= 1e-10, (b, errs)
            follows[b] = alt
    pm_ref = np.stack([follows[b]["pmean"][b] for b in range(B)])
    pv_ref = np.stack([follows[b]["pvar"][b] for b in range(B)])
    assert np.abs(pm - pm_ref).max() <= 1.3e-6 * np.abs(pm_ref).max()
    assert (np.abs(pv - pv_ref) / kxx).max() <= 1e-8
