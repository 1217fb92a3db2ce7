"""Benchmark: GP fit+predict points/sec at n = 2^20, fp64 (BASELINE.json metric) on MI355X.

Workload (BASELINE config C4 "FastGPLattice n=2^20 d=5, 64 random shifts batched
across 8 MI355X"): every rank owns `--shifts` independent randomly shifted lattice GPs (weak
scaling: 8 per GPU -> 64 at N=8; seeds 1000 + global shift index).  One step = for every shift:
  y~ = ft(y), k1 parts, fit (K=50 Rprop iterations, early stopping disabled), coeffs = K^-1 y,
  post_mean at N=256 test points, post_var at N=8 test points.
Inputs (points, y = f_ackley(x)) are resident in HBM before the timed region; GP state is reset to the
initial hyper-parameters and all caches are dropped at the start of every step.
value = (shifts * n * world_size) / (max-over-ranks seconds per step).

Extra JSON keys: "roofline" for the dominant kernel (priced on the rocprofv3 kernel-trace average of this
command committed under profiles/; its launches also timed live on the device clock, fgp_nll_desc.stamps,
and with HIP events, both reported beside it),
"cpu_baseline" (the oracle = torch-CPU restatement of the reference, rank 0 at N=1, bounded sample),
"phases_ms" (per-phase breakdown of one batched step, HIP events).
"""
import argparse
import json
import math
import os
import time

import numpy as np
import torch

torch.set_default_dtype(torch.float64)

from benchkit.common import FP64_PEAK_TFS, HBM_PEAK_GBS, _clear_capture_error, f_ackley  # noqa: F401
from benchkit.extras import (  # noqa: F401
    PAPER_S_PER_STEP, paper_functions, f_grad_f, paper_configs, multitask_configs, batch_multitask_configs
)
from benchkit.pricing import (  # noqa: F401
    STAGES, SPEC_BLOCKS, stage_names, spec_tile_geometry, spec_geometry, spec_tile_grid, spec_fused, r2c_active,
    fit_variant, re_row_log2, fit_grid, stage_bytes, wall_clock_khz, roofline_fit_kernels, graph_fit_us, ROOT,
    PMC_SUMMARY, PMC_SQ_SUMMARY, ROCPROF_GRID_STATS, STREAM_FLOOR_US, FP64_LANE_OPS_PEAK, CPU_FIDELITY,
    ROCPROF_PREDICT_STATS, PMC_SQ_PREDICT, pmc_traffic, _kernel_match, pmc_valu_insts, rocprof_avg_us,
    post_mean_ops_per_pair, roofline_post_mean, SECONDARY_STATS, FP64_MFMA_PEAK_FLOPS, secondary_rooflines
)



def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    p.add_argument("--shifts", type=int, default=8, help="independent GPs per GPU")
    p.add_argument("--fit-iters", type=int, default=50)
    p.add_argument("--n-mean", type=int, default=256)
    p.add_argument("--n-var", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--sequential", dest="batched", action="store_false",
                   help="fit and predict the shifts one by one (default: one GPBatch over all shifts)")
    p.add_argument("--cpu-sample-iters", type=int, default=3)
    p.add_argument("--no-secondary", dest="secondary", action="store_false",
                   help="skip the secondary BASELINE configs (C2, C3, C5) reported under 'secondary'")
    p.add_argument("--c5-outputs", type=int, default=512)
    p.add_argument("--no-graph", dest="graph", action="store_false",
                   help="time the eager enqueue of each step instead of replaying its hipGraph capture")
    p.add_argument("--no-multitask", dest="multitask", action="store_false",
                   help="skip the docs/examples/multitask per-step timings reported under 'multitask'")
    p.add_argument("--no-paper", dest="paper", action="store_false",
                   help="skip the probnum25 paper's n=2^10 per-step timings reported under 'paper'")
    p.add_argument("--dump", default=None,
                   help="directory: every rank writes its shifts' seeds, fitted raw parameters, post_mean and post_var "
                        "after the timed steps to rank<r>.npz (the N-rank test compares them with N = 1 runs)")
    return p.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`bench.py --gpus N` (N > 1) started without a launcher: run torch.distributed.run with N ranks over this
    same command line as a CHILD process -- before this process makes any GPU call -- relay rank 0's JSON line
    and return the child's exit code.  (The driver's own N-GPU runs start under torch.distributed.run, with
    WORLD_SIZE set, and go straight to main.)"""
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    for line in proc.stdout:
        if line.startswith("{"):
            print(line.rstrip("\n"), flush=True)
        else:
            sys.stderr.write(line)
    return proc.wait()


def shard_seeds(rank, world, per_rank, base=1000):
    """Replica sharding of the C4 shifts: rank r owns global shifts r*per_rank ... (weak scaling);
    no data-path collective (independent GPs)."""
    return [base + rank * per_rank + s for s in range(per_rank)]


def max_over_ranks(seconds, device):
    """Max of the per-rank elapsed time (the only collective: timing, not data)."""
    import torch.distributed as tdist
    if not (tdist.is_available() and tdist.is_initialized()) or tdist.get_world_size() == 1:
        return seconds
    if tdist.get_backend() == "gloo":
        device = "cpu"              # gloo reduces host tensors (the CPU / one-GPU multi-process tests)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t)


class Shifts(object):
    """The rank's randomly shifted lattice GPs with resident inputs: points (generated once, untimed),
    observations y [P, n] and the initial raw hyper-parameters [P, 2 + d] in HBM."""

    def __init__(self, F, d, n, seeds, device):
        self.gps, ys = [], []
        for seed in seeds:
            gp = F.FastGPLattice(F.Lattice(d, seed=seed, randomize="SHIFT"), device=device)
            x = gp.get_x_next(n)                         # host point generation: untimed
            y = f_ackley(x).contiguous()
            gp.add_y_next(y)
            self.gps.append(gp)
            ys.append(y)
        self.y = torch.stack(ys)
        self.batch = F.GPBatch(self.gps)
        self.raw0 = self.batch.raw().clone()
        self.n = n

    def reset(self):
        """Fresh start of a step: initial hyper-parameters, the observations re-ingested, every cache
        (ytilde, parts, coefficients) dropped."""
        self.batch.set_data(self.y)
        self.batch.set_raw(self.raw0.clone())


def step_batched(sh, args, xm, xv, store_loss_hist=False):
    """One timed step; returns (per-GP fit data, post_mean [P, N], post_var [P, N]) so the parity
    test (tests/test_gpu_bench_path.py) checks exactly this sequence.  store_loss_hist only copies the
    device loss history back after the fit (the device work is the same)."""
    sh.reset()
    data = sh.batch.fit(iterations=args.fit_iters, stop_crit_wait_iterations=args.fit_iters + 1,
                        store_loss_hist=store_loss_hist)
    pm = sh.batch.post_mean(xm)
    pv = sh.batch.post_var(xv)
    return data, pm, pv


def step_sequential(sh, args, xm, xv):
    sh.reset()
    for gp in sh.gps:
        gp.fit(iterations=args.fit_iters, stop_crit_wait_iterations=args.fit_iters + 1, verbose=0)
        gp.post_mean(xm)
        gp.post_var(xv)


class SingleGP(object):
    """BASELINE configs C2 / C3: one fast GP of n = 2^16, d = 3 (lattice / digital net with the
    reference's default alpha = 2), inputs resident; reset = fresh data ingest + initial parameters."""

    def __init__(self, F, family, log2n, d, device):
        n = 2 ** log2n
        if family == "lattice":
            self.gp = F.FastGPLattice(F.Lattice(d, seed=7), device=device)
        else:
            self.gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=7), device=device)
        self.y = f_ackley(self.gp.get_x_next(n)).contiguous()
        self.raw0 = [p.detach().clone() for p in (self.gp.raw_scale, self.gp.raw_lengthscales, self.gp.raw_noise)]
        self.n, self.outputs = n, 1

    def reset(self):
        gp = self.gp
        gp._y[0] = gp._y[0][..., :0]
        gp._nh = 0
        gp.add_y_next(self.y)
        # fresh initial parameters: one copy of the three, each a Parameter over its slice
        flat = torch.cat([v.reshape(-1) for v in self.raw0])
        o = 0
        for name, v in zip(("raw_scale", "raw_lengthscales", "raw_noise"), self.raw0):
            old = getattr(gp, name)
            setattr(gp, name, torch.nn.Parameter(flat[o:o + v.numel()].view(v.shape), requires_grad=old.requires_grad))
            o += v.numel()
        gp._cache, gp._snap = {}, None


class MultiOutputGP(SingleGP):
    """BASELINE config C5: one FastGPLattice, n = 2^18, d = 3, shape_batch = [B] outputs,
    y_b = f_ackley(x) (1 + b / B) + 0.01 randn (seeded; the [B, n] noise is drawn whole and sliced, so an
    output's data do not depend on the rank that owns it).  Shared hyper-parameters (the reference's
    default shape_scale = [1], shape_lengthscales = [d]), or per_output ones
    (shape_scale = [B, 1], shape_lengthscales = [B, d]: B independent eigen-problems on one point set,
    docs/examples/batch_multitask/fgp_lattice.ipynb cell 6).  `shard` = (start, stop): the outputs this
    rank owns (bench.py under torchrun).  fp64 (the reference's precision) or fp32 observations."""

    def __init__(self, F, log2n, d, outputs, device, data_dtype=torch.float64, shard=None, per_output=False):
        n = 2 ** log2n
        a, b = shard if shard is not None else (0, outputs)
        B = b - a
        extra = dict(shape_scale=[B, 1], shape_lengthscales=[B, d]) if per_output else {}
        self.gp = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[B], device=device, data_dtype=data_dtype, **extra)
        # the observations formed on the host (untimed set-up) exactly as tests/golden/make_golden_c5.py's c5_data, so the
        # benched data are the REAL reference's fixture inputs bit for bit (tests/test_gpu_multioutput.py)
        f = f_ackley(self.gp.get_x_next(n).cpu())
        g = torch.Generator().manual_seed(5)
        noise = torch.randn((outputs, n), generator=g, dtype=torch.float64)
        bb = torch.arange(outputs, dtype=torch.float64)[:, None]
        self.y = (f[None, :] * (1 + bb / outputs) + 0.01 * noise)[a:b].to(data_dtype).contiguous().to(device)
        del noise
        self.raw0 = [p.detach().clone() for p in (self.gp.raw_scale, self.gp.raw_lengthscales, self.gp.raw_noise)]
        self.n, self.outputs, self.total = n, B, outputs
        self.sharded = shard is not None and B < outputs and not per_output


def step_single(sg, args, xm, xv):
    """One step of a single GP (C2, C3) or of a multi-output GP (C5): fresh data, fit, post_mean, post_var.
    A C5 GP whose outputs are sharded over the ranks fits with distributed.fit_sharded (ONE all-reduce of
    Y = sum_b |ytilde_b|^2, then the identical fit on every rank)."""
    sg.reset()
    its = dict(iterations=args.fit_iters, stop_crit_wait_iterations=args.fit_iters + 1)
    if getattr(sg, "sharded", False):
        from fastgaussianprocesses_amd.distributed import fit_sharded
        fit_sharded(sg.gp, sg.total, **its)
    else:
        sg.gp.fit(verbose=0, **its)
    pm = sg.gp.post_mean(xm)
    pv = sg.gp.post_var(xv)
    return pm, pv


def fit_graph_stats(F):
    """fgp_fit_graph_stats: [replays of a cached fit graph, captures, eager fallbacks] since the library loaded."""
    import ctypes
    out = (ctypes.c_longlong * 3)()
    F._native.call("fgp_fit_graph_stats", out)
    return list(out)


def persist_giveups(F):
    """The library's sticky count of single-launch-fit barrier give-ups (fgp_persist_giveups; synchronises)."""
    return F.fit_engine.persist_giveups()


def replay_giveup_error(F, before):
    """None, or the message of fit_engine.check_replayed_fits when a single-launch fit gave up since `before`."""
    try:
        F.fit_engine.check_replayed_fits(before)
        return None
    except RuntimeError as e:
        return str(e)


def time_steps(fn, steps, warmup, device=None):
    """Seconds per step: warmup, then `steps` steps bracketed by a barrier + device sync on both sides,
    the max over the ranks when a process group is up."""
    import torch.distributed as tdist
    dist = tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    el = time.perf_counter() - t0
    if dist:
        el = max_over_ranks(el, device)
    return el / steps


def total_outputs(sg):
    return getattr(sg, "total", 1)


def c5_shard(outputs, rank, world):
    from fastgaussianprocesses_amd.distributed import output_shard
    return output_shard(outputs, rank, world) if world > 1 else None


def secondary_configs(F, args, device, rank=0, world=1, collect=None):
    """The other BASELINE.json configs, each timed as its own step (fit K Rprop iterations without early
    stopping + post_mean N + post_var N):
      N = 1 only: C2 FastGPLattice n=2^16 d=3, C3 FastGPDigitalNetB2 n=2^16 d=3 (default alpha = 2), C5 with
        fp32 observations;
      every N (all ranks take part, max-over-ranks time, value = all outputs x n / s): C5 multi-output
        FastGPLattice n=2^18 d=3 x B outputs, fp64, outputs sharded over the ranks (fit_sharded: one Y
        all-reduce), and C5 with per-output hyper-parameters (B independent eigen-problems; replicas, no
        collective).
    collect: a dict that receives, per case ("C2", "C5", "C5 per-output", ...), one more step's fitted raw
    parameters, post_mean and post_var (host tensors) and the outputs this rank owns --
    tests/test_gpu_multioutput.py compares the N = 2 lines' with the N = 1 run's."""
    B = args.c5_outputs
    sh = c5_shard(B, rank, world)
    cases = []
    if world == 1:
        cases += [("C2: FastGPLattice n=2^16 d=3", lambda: SingleGP(F, "lattice", 16, 3, device), 3),
                  ("C3: FastGPDigitalNetB2 n=2^16 d=3 alpha=2", lambda: SingleGP(F, "net", 16, 3, device), 3)]
    cases.append(("C5: FastGPLattice n=2^18 d=3 x %d outputs (shared hyper-parameters), fp64%s"
                  % (B, ", outputs sharded over %d ranks (one Y all-reduce)" % world if world > 1 else ""),
                  lambda: MultiOutputGP(F, 18, 3, B, device, shard=sh), 3))
    cases.append(("C5 per-output: FastGPLattice n=2^18 d=3 x %d outputs, per-output hyper-parameters "
                  "(shape_scale=[%d,1], shape_lengthscales=[%d,3]), fp64%s"
                  % (B, B, B, ", replicas over %d ranks" % world if world > 1 else ""),
                  lambda: MultiOutputGP(F, 18, 3, B, device, shard=sh, per_output=True), 3))
    if world == 1:
        cases.append(("C5 mixed: FastGPLattice n=2^18 d=3 x %d outputs, fp32 observations widened on load into "
                      "one fp64 half-spectrum transform (Y and coefficients), fp64 eigenvalues / posteriors" % B,
                      lambda: MultiOutputGP(F, 18, 3, B, device, torch.float32), 3))
    out = []
    for name, make, d in cases:
        sg = make()
        g = torch.Generator().manual_seed(17)      # per case: the same test points at every N
        xm = torch.rand((args.n_mean, d), generator=g).to(device)
        xv = torch.rand((args.n_var, d), generator=g).to(device)
        # the median of 3 windows of >= 5 timed steps (each bracketed as time_steps does) after 2 warm-ups: a
        # one-off host stall (allocator growth, a page fault) in a ~1 ms step is not the config's rate
        one = lambda: step_single(sg, args, xm, xv)
        graph, ginfo = None, {"used": False}
        if world == 1 and getattr(args, "graph", False):
            for _ in range(2):
                one()
            graph, ginfo = capture_fn(one)
        run = graph.replay if graph is not None else one
        gu0 = persist_giveups(F)
        wins = sorted(time_steps(run, max(5, args.steps), 2 if w == 0 else 0, device) for w in range(3))
        sec = wins[1]
        # a single-launch fit that gave up inside a timed replay (its control word cannot be read in a capture) would
        # have timed NaN parameters: the library's sticky give-up count must not have moved (fails the line)
        giveup_err = replay_giveup_error(F, gu0)
        if graph is not None:
            ginfo["eager_ms_per_step"] = sorted(time_steps(one, max(5, args.steps), 0, device)
                                                for _ in range(3))[1] * 1e3
        if collect is not None:
            pm, pv = step_single(sg, args, xm, xv)
            collect[name.split(":")[0]] = dict(
                raw_scale=sg.gp.raw_scale.detach().cpu().clone(),
                raw_lengthscales=sg.gp.raw_lengthscales.detach().cpu().clone(),
                post_mean=pm.detach().cpu().clone(), post_var=pv.detach().cpu().clone(),
                outputs=c5_shard(total_outputs(sg), rank, world) if world > 1 else (0, total_outputs(sg)))
        phases = None
        if world == 1:
            # per-phase median of 3 event-timed steps (one sample can catch a host stall)
            keys = ("ytilde+fit", "coeffs", "post_mean", "post_var")
            samples = []
            for _ in range(3):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
                sg.reset()
                ev[0].record()
                sg.gp.fit(iterations=args.fit_iters, stop_crit_wait_iterations=args.fit_iters + 1, verbose=0)
                ev[1].record()
                with torch.no_grad():
                    sg.gp.coeffs                 # the graph-free coefficients post_mean uses
                ev[2].record()
                sg.gp.post_mean(xm)
                ev[3].record()
                sg.gp.post_var(xv)
                ev[4].record()
                torch.cuda.synchronize()
                samples.append([ev[i].elapsed_time(ev[i + 1]) for i in range(4)])
            phases = {k: sorted(s[i] for s in samples)[1] for i, k in enumerate(keys)}
            if graph is not None:
                ginfo["phases_ms"] = graph_phases(F, sg, args, xm, xv, device)
        total = getattr(sg, "total", 1)
        roof_pm = None
        if name.startswith("C5 per-output"):
            # 512 outputs with their own kernels: k_post_mean<0, 3, 4, 4> over the outputs in blocks of 4, ONE launch
            # (fgp_post_mean over output blocks: N x n x 4 output-pairs per block, B / 4 blocks), priced on
            # tools/predict_kernels.py's trace of the same call
            roof_pm = roofline_post_mean("k_post_mean<0, 3, 4, 4>", None, args.n_mean * sg.n * 4 * (sg.outputs // 4), 3, 4,
                                         stats=ROCPROF_PREDICT_STATS, sq=PMC_SQ_PREDICT,
                                         live_ms=phases.get("post_mean") if phases else None,
                                         launches=1 + (1 if sg.outputs % 4 else 0))
        roofs = secondary_rooflines(name.split(":")[0], sg.n, d, total, args.n_mean, args.fit_iters)
        out.append({"metric": "GP fit+predict points/sec" if total == 1 else
                    "multi-output GP fit+predict output-points/sec",
                    "roofline": roofs[0] if roofs else None, "rooflines_other": roofs[1:],
                    "value": None if giveup_err else sg.n * total / sec, "error": giveup_err,
                    "unit": "points/s" if total == 1 else "output-points/s",
                    "ms_per_step": sec * 1e3, "steps": max(5, args.steps), "n_gpus": world,
                    "dtype": "f64" if sg.gp.data_dtype == torch.float64 else "f32 data / f64 eigenvalues",
                    "config": {"workload": "%s: fit %d Rprop iters + post_mean N=%d + post_var N=%d"
                                           % (name, args.fit_iters, args.n_mean, args.n_var),
                               "n": sg.n, "outputs": total},
                    "phases_ms": phases, "graph": ginfo, "roofline_predict": roof_pm})
        del graph, sg
        torch.cuda.empty_cache()
    return out


def phase_breakdown(sh, iters, xm, xv):
    """HIP-event timing of each phase of one batched step over the rank's shifts (torch's current
    stream)."""
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
    sh.reset()
    b = sh.batch
    ev[0].record()
    b.ysq()
    ev[1].record()
    b.basis()          # part-product spectra (spectral fit path; None on the transform path)
    ev[2].record()
    b.fit(iterations=iters, stop_crit_wait_iterations=iters + 1)
    ev[3].record()
    b.coeffs()
    ev[4].record()
    b.post_mean(xm)
    ev[5].record()
    b.post_var(xv)
    ev[6].record()
    torch.cuda.synchronize()
    names = ["ytilde", "basis", "fit", "coeffs", "post_mean", "post_var"]
    return {names[i]: ev[i].elapsed_time(ev[i + 1]) for i in range(6)}


def cpu_baseline(args, n, d):
    """Oracle (torch-CPU restatement of the reference) on a bounded sample of one GP, scaled to the
    per-GP workload of one step."""
    from oracle import fgp_oracle as O
    torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    threads = torch.get_num_threads()
    seq = np.random.default_rng(1000).uniform(size=d)
    from fastgaussianprocesses_amd.seqs import DEFAULT_LATTICE_Z
    x = torch.from_numpy(O.lattice_points(DEFAULT_LATTICE_Z[:d], seq, 0, n))
    y = f_ackley(x)
    o = O.OracleFastGP("lattice", x, None, y, alpha=2)
    t0 = time.perf_counter()
    o.ytilde()
    o.k1parts()
    t_setup = time.perf_counter() - t0
    k = args.cpu_sample_iters
    t0 = time.perf_counter()
    o.fit(iterations=k, stop_crit_wait_iterations=k + 1)
    t_fit_per = (time.perf_counter() - t0) / (k + 1)   # k+1 loss evaluations, k backward+steps
    t0 = time.perf_counter()
    o.coeffs()
    t_coeffs = time.perf_counter() - t0
    g = torch.Generator().manual_seed(17)
    nm = 8
    xm = torch.rand((nm, d), generator=g)
    t0 = time.perf_counter()
    o.post_mean(xm, chunk=4)
    t_pm = (time.perf_counter() - t0) / nm
    xv = torch.rand((1, d), generator=g)
    t0 = time.perf_counter()
    o.post_var(xv)
    t_pv = time.perf_counter() - t0
    t_gp = t_setup + (args.fit_iters + 1) * t_fit_per + t_coeffs + args.n_mean * t_pm + args.n_var * t_pv
    try:    # oracle / reference timed on the same cores in the build container
        fid = json.load(open(CPU_FIDELITY))["port_vs_reference"]
    except (OSError, ValueError, KeyError):
        fid = None
    return {"value": n / t_gp, "unit": "points/s", "cores": threads, "kind": "port",
            "port_vs_reference": fid, "port_vs_reference_source": os.path.relpath(CPU_FIDELITY, ROOT),
            "sample": ("oracle (oracle/fgp_oracle.py, torch-CPU restatement of the reference) on one n=2^%d d=%d GP: "
                       "ytilde+parts, %d fit iterations, coeffs, post_mean of %d points, post_var of 1 point; scaled "
                       "to %d fit iterations + post_mean N=%d + post_var N=%d per GP" %
                       (int(math.log2(n)), d, k, nm, args.fit_iters, args.n_mean, args.n_var)),
            "seconds_per_gp": t_gp}


def graph_phases(F, sg, args, xm, xv, device, reps=5):
    """Device time of each phase of a single-GP / multi-output step REPLAYED from a hipGraph: the step captured
    with a device-clock stamp kernel (fgp_clock_stamp) between its phases (ytilde+fit, coeffs, post_mean,
    post_var), replayed `reps` times, the median of the stamp differences per phase (ms).  The eager
    `phases_ms` also hold the host's enqueue time; these do not (each stamp adds one ~2 us launch).  None when
    the capture fails."""
    st = torch.zeros(5, dtype=torch.int64, device=device)
    call = F._native.call

    def stamp(i):
        call("fgp_clock_stamp", st[i:i + 1].data_ptr(), torch.cuda.current_stream().cuda_stream)

    def fn():
        sg.reset()
        stamp(0)
        sg.gp.fit(iterations=args.fit_iters, stop_crit_wait_iterations=args.fit_iters + 1, verbose=0)
        stamp(1)
        with torch.no_grad():
            sg.gp.coeffs
        stamp(2)
        pm = sg.gp.post_mean(xm)
        stamp(3)
        pv = sg.gp.post_var(xv)
        stamp(4)
        return pm, pv
    g, info = capture_fn(fn)
    if g is None:
        return None
    khz = wall_clock_khz(F, torch.device(device))
    rows = []
    for _ in range(reps):
        g.replay()
        torch.cuda.synchronize()
        t = st.cpu().tolist()
        rows.append([(t[i + 1] - t[i]) / khz for i in range(4)])
    keys = ("ytilde+fit", "coeffs", "post_mean", "post_var")
    return {k: sorted(r[i] for r in rows)[reps // 2] for i, k in enumerate(keys)}


def capture_fn(fn):
    """fn() (returning a tuple of device tensors) captured once into a hipGraph; (graph, info).  The replay's
    outputs must equal an eager call's bit for bit, else (None, info) and the caller times the eager calls."""
    info = {"used": False}
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # thread-local capture mode on an explicit stream (every phase captures cleanly this way,
        # tools/diag_capture.py, removed in round 6: git show 1846d2f:tools/diag_capture.py)
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                out = fn()
                if os.environ.get("FGP_BENCH_GRAPH_FAIL") == "1":      # test hook: the eager fallback
                    torch.cuda.synchronize()                          # (a sync inside a capture invalidates it)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        got = [t.clone() for t in out]
        ref = fn()
        torch.cuda.synchronize()
        if not all(torch.equal(a, b) for a, b in zip(got, ref)):
            info["error"] = "replay differs from the eager call"
            return None, info
        info.update({"used": True, "check": "replay == eager call (post_mean, post_var bit for bit)"})
        return g, info
    except Exception as e:          # capture not possible here: time the eager enqueue
        import traceback
        info["error"] = repr(e)[:300]
        info["where"] = [ln.strip() for ln in traceback.format_exc().splitlines() if "repo" in ln][-4:]
        _clear_capture_error()
        return None, info


def capture_step(sh, args, xm, xv):
    """The whole batched step (data re-ingest + parameter reset, ytilde, spectra, 50 fit iterations, coefficients,
    post_mean, post_var) captured once into a hipGraph and replayed per timed step: the same device work,
    without the host's per-launch Python.  Checked on the spot: a replay's post_mean / post_var equal an eager
    step's bit for bit, else the eager loop is timed (graph_info says why)."""
    return capture_fn(lambda: step_batched(sh, args, xm, xv)[1:])


def main():
    import sys
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test overrides: every rank on one device (FGP_BENCH_DEVICE) and the gloo backend (the N-rank test on one GPU)
    if os.environ.get("FGP_BENCH_DEVICE"):
        local = int(os.environ["FGP_BENCH_DEVICE"])
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        backend = os.environ.get("FGP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    import fastgaussianprocesses_amd as F
    n = 2 ** args.log2n
    d = args.d
    shifts = Shifts(F, d, n, shard_seeds(rank, world, args.shifts), device)
    g = torch.Generator().manual_seed(17)
    xm = torch.rand((args.n_mean, d), generator=g).to(device)
    xv = torch.rand((args.n_var, d), generator=g).to(device)

    def step():
        (step_batched if args.batched else step_sequential)(shifts, args, xm, xv)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    graph, graph_info = None, {"used": False}
    if args.graph and args.batched:
        graph, graph_info = capture_step(shifts, args, xm, xv)
    # two device-clock stamp kernels bracket the timed loop (outside the timed interval): the first two
    # k_clock_stamp launches of a rocprofv3 --kernel-trace of this command mark the timed region, whose launches
    # tools/timed_region_stats.py averages (the graph replays' per-kernel durations the roofline is priced on)
    gu0 = persist_giveups(F)
    marks = torch.zeros(2, dtype=torch.int64, device=device)
    F._native.call("fgp_clock_stamp", marks[0:1].data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if graph is not None:
            graph.replay()
        else:
            step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, device)
    F._native.call("fgp_clock_stamp", marks[1:2].data_ptr(), torch.cuda.current_stream().cuda_stream)
    sec_step = el / args.steps
    value = args.shifts * n * world / sec_step
    giveup_err = replay_giveup_error(F, gu0)
    if giveup_err:
        raise RuntimeError("timed steps invalid: " + giveup_err)
    if graph is not None:
        # the same steps enqueued eagerly (host-side Python per launch), for comparison
        torch.cuda.synchronize()
        gs0 = fit_graph_stats(F)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        graph_info["eager_ms_per_step"] = (time.perf_counter() - t0) / args.steps * 1e3
        graph_info["eager_fit_graphs"] = dict(zip(("replays", "captures", "eager"),
                                                  [b - a for a, b in zip(gs0, fit_graph_stats(F))]))

    if args.dump:
        # one more step's results (every step is the same computation from the same reset state)
        data, pm, pv = step_batched(shifts, args, xm, xv)
        torch.cuda.synchronize()
        os.makedirs(args.dump, exist_ok=True)
        np.savez(os.path.join(args.dump, "rank%d.npz" % rank), seeds=np.array(shard_seeds(rank, world, args.shifts)),
                 raw=shifts.batch.raw().cpu().numpy(), post_mean=pm.cpu().numpy(), post_var=pv.cpu().numpy())
    phases = phase_breakdown(shifts, args.fit_iters, xm, xv)
    n_, variant, us, us_ev, t_iter, khz = roofline_fit_kernels(F, shifts, args.fit_iters)
    parts_array = variant not in ("spectral", "spectral_fused", "re")
    P = len(shifts.gps)
    sb = stage_bytes(n, d, P, parts_array, variant)
    dom = max(stage_names(variant), key=lambda k: us[k])
    kname = dom + {"re": "_re", "r2c": "_r2c", "full": "", "spectral": "", "spectral_fused": ""}[variant]
    grid_wg, wg_thr = fit_grid(n, P, variant, d)[dom]
    # achieved / frac are priced on the rocprofv3 kernel-trace average of this same command (committed
    # under profiles/) when it is there -- the duration the profiler reports, including the dispatch
    # ramp; the live device-clock figure (first workgroup start to last wave end) is reported beside it
    us_rp = rocprof_avg_us(kname, grid_wg * wg_thr)
    us_price = us_rp if us_rp is not None else us[dom]
    ach = sb[dom] / (us_price * 1e-6) / 1e9
    roof = {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": pmc_traffic(kname, grid_wg * wg_thr),
            "traffic_source": os.path.relpath(PMC_SUMMARY, ROOT),
            "algorithmic_bytes": sb[dom],
            "avg_us": us_price, "avg_us_source": ("rocprofv3 --kernel-trace of this bench command, the launches "
                                                  "inside its timed region (graph replays; tools/timed_region_stats.py), %s"
                                                  % os.path.relpath(ROCPROF_GRID_STATS, ROOT))
            if us_rp is not None else "device clock (live)",
            "avg_us_device_clock": us[dom], "avg_us_device_clock_source": "this run: device clock (%d kHz), "
            "first workgroup start to last wave end, mean of %d launches" % (khz, args.fit_iters),
            "frac_device_clock": sb[dom] / (us[dom] * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "avg_us_events": us_ev[dom],
            "avg_us_graph_events": us_ev.get(dom + "@graph"),
            "avg_us_graph_events_source": "this run: HIP events around hipGraph replays of the fit's launch sequence "
                                          "(fgp_fit_run captured, as in the timed step), per iteration",
            "launch": "%d problems x n=2^%d (grid %d workgroups)" % (P, args.log2n, grid_wg),
            "transform": {"re": "real-even: n/2-point transform, columns [0, N2/2) (n/4 complex)",
                          "r2c": "half-length R2C (n/2 complex)", "full": "full-length (n complex)",
                          "spectral": "none per iteration: lambda from the 2^d part-product spectra",
                          "spectral_fused": "none per iteration: lambda from the 2^d part-product spectra; "
                                            "the kernel also reduces the partials (two deterministic levels) "
                                            "and applies every problem's Rprop step"}[variant],
            "kernels": {k: {"avg_us": us[k], "avg_us_events": us_ev[k], "bytes": sb.get(k),
                            "GB/s": (sb[k] / (us[k] * 1e-6) / 1e9) if k in sb else None} for k in us},
            "parts": ("spectra (fgp_spec_basis, built in the step)" if variant.startswith("spectral") else
                      "array" if parts_array else "regenerated (FGP_PARTS_LATTICE)"),
            "iteration_us": t_iter * 1e6}
    vi = pmc_valu_insts(kname, grid_wg * wg_thr)
    if vi is not None:
        # the same kernel against the FP64 VALU issue peak, on the SAME duration as `frac` (avg_us).  Every
        # VALU instruction priced as a 64-lane FP64 one (integer / FP32 ones issue faster): an upper
        # estimate of the issue-slot use.
        lane_ops = vi * 64 / (us_price * 1e-6)
        roof["valu"] = {"insts_per_launch": vi, "lane_ops_per_s": lane_ops, "peak_fp64_lane_ops_per_s": FP64_LANE_OPS_PEAK,
                        "frac": lane_ops / FP64_LANE_OPS_PEAK, "time": "avg_us",
                        "source": os.path.relpath(PMC_SQ_SUMMARY, ROOT) + " (SQ_INSTS_VALU)"}
    if variant.startswith("spectral"):
        # what the dataflow of the reference would move per iteration (B_iter = 16nd + 32n +
        # 32n bytes per GP -- parts read twice, lambda written and re-read, ytilde read twice) is NOT a bound
        # for this path: the spectral iteration reads only the shared spectra and Y (algorithmic_bytes)
        b_iter = (16 * n * d + 64 * n) * P
        roof["survey_byte_model"] = {
            "bytes_per_iteration": b_iter, "effective_GBps": b_iter / (us_price * 1e-6) / 1e9,
            "note": "SURVEY 8(d) reference-dataflow bytes over the kernel's duration; not a bound of the spectral "
                    "path, which reads only the 2^d shared spectra and Y per iteration"}
        roof["read_floor"] = {"us": STREAM_FLOOR_US, "frac": STREAM_FLOOR_US / us_price,
                              "source": "tools/stream_microbench.hip, profiles/r03v_stream_and_stamps.jsonl"}
    # the posterior mean (about a third of the step): FP64-VALU roofline of its one k_post_mean launch over the P
    # shifts (fgp_post_mean_batched), priced on the same rocprofv3 trace as `roofline`
    roof_pm = roofline_post_mean("k_post_mean<0, %d, 1, 4>" % d, None, P * args.n_mean * n, d, 1, sq=PMC_SQ_PREDICT,
                                 live_ms=phases.get("post_mean"))
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # after the timed region on every N (rank 0 only; the other ranks wait at the next collective), so the
        # N-GPU line carries the CPU baseline beside its scaling
        cpu = cpu_baseline(args, n, d)
    secondary = None
    if args.secondary:
        secondary = secondary_configs(F, args, device, rank, world)
    paper = None
    if args.paper and world == 1:
        paper = {"source": "docs/examples/probnum25_paper/benchmarks_accuracy_time.tex:6-10 (time per optimization "
                           "step, s; the paper's hardware is unstated) with the protocol of probnum25_paper.ipynb "
                           "cell 15 (fit wall time / iterations, reference fit defaults)",
                 "configs": paper_configs(F, device)}
    multitask = None
    if args.multitask and world == 1:
        multitask = multitask_configs(F, device)
    if rank == 0:
        out = {"metric": "GP fit+predict points/sec at n=2^20 fp64; achieved HBM GB/s vs roofline",
               "value": value, "unit": "points/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": sec_step * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "f64", "data": "synthetic (f_ackley on shifted rank-1 lattices)",
               "config": {"workload": "C4: FastGPLattice n=2^%d d=%d, %d random shifts per GPU, fit %d Rprop iters + "
                                      "post_mean N=%d + post_var N=%d per shift" %
                                      (args.log2n, d, args.shifts, args.fit_iters, args.n_mean, args.n_var),
                          "global_shifts": args.shifts * world, "parallelism": "replicas%d" % world},
               "timing": {"value_from": "hipGraph replay of the whole step (captured once, replay checked bit-identical "
                                        "to an eager step)" if graph is not None else "eager enqueue of every step",
                          "value_eager": (args.shifts * n * world / (graph_info["eager_ms_per_step"] * 1e-3)
                                          if graph is not None else value),
                          "ms_per_step_eager": graph_info.get("eager_ms_per_step", sec_step * 1e3)},
               "roofline": roof, "roofline_predict": roof_pm,
               "cpu_baseline": cpu, "phases_ms": phases, "secondary": secondary,
               "paper": paper, "multitask": multitask, "graph": graph_info}
        print(json.dumps(out))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
