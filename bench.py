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

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6           # MI355X FP64 vector/matrix peak (spec)


def f_ackley(x, a=20, b=0.2, c=2 * np.pi, scaling=32.768):
    # the reference's doctest workload (fastgps/fast_gp_lattice.py:14-22)
    x = 2 * scaling * x - scaling
    t1 = a * torch.exp(-b * torch.sqrt(torch.mean(x ** 2, 1)))
    t2 = torch.exp(torch.mean(torch.cos(c * x), 1))
    return -t1 - t2 + a + np.exp(1)


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
        for name, v in zip(("raw_scale", "raw_lengthscales", "raw_noise"), self.raw0):
            old = getattr(gp, name)
            setattr(gp, name, torch.nn.Parameter(v.clone(), requires_grad=old.requires_grad))
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


# ---------------------------------------------------------------- the probnum25 paper's timing table
# docs/examples/probnum25_paper/benchmarks_accuracy_time.tex:6-10 ("time per optimization step", seconds; the
# paper's hardware is unstated): {benchmark: (SI lattice f, SI lattice (f, grad f), DSI net f, DSI net (f, grad f))}
PAPER_S_PER_STEP = {"Ackley": (5.6e-4, 1.3e-3, 7.7e-4, 1.9e-3), "Branin": (5.3e-4, 2.1e-3, 7.0e-4, 3.4e-3),
                    "Camel": (5.0e-4, 2.2e-3, 6.8e-4, 3.4e-3), "StyTang": (5.2e-4, 2.2e-3, 7.7e-4, 3.4e-3),
                    "Hartmann": (5.1e-4, 8.3e-3, 7.1e-4, 1.6e-2)}


def paper_functions():
    """The paper's benchmark functions (probnum25_paper.ipynb cell 7; the standard test-function
    definitions) as (name, d, f, Baker transform for the lattice's (f, grad f) fit) -- cell 15's `funcs`."""
    def branin(x):
        a, b, c, r, s, t = 1.0, 5.1 / (4 * np.pi ** 2), 5 / np.pi, 6.0, 10.0, 1 / (8 * np.pi)
        x1, x2 = 15 * x[:, 0] - 5, 15 * x[:, 1]
        return a * (x2 - b * x1 ** 2 + c * x1 - r) ** 2 + s * (1 - t) * torch.cos(x1) + s

    def camel(x):
        x1, x2 = 6 * x[:, 0] - 3, 4 * x[:, 1] - 2
        return (4 - 2.1 * x1 ** 2 + x1 ** 4 / 3) * x1 ** 2 + x1 * x2 + (-4 + 4 * x2 ** 2) * x2 ** 2

    def styblinski_tang(x):
        x = 10 * x - 5
        return 0.5 * torch.sum(x ** 4 - 16 * x ** 2 + 5 * x, 1)

    def hartmann(x):
        al = torch.tensor([1.0, 1.2, 3.0, 3.2], device=x.device)
        A = torch.tensor([[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14], [3, 3.5, 1.7, 10, 17, 8],
                          [17, 8, 0.05, 10, 0.1, 14]], device=x.device)
        P = 1e-4 * torch.tensor([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                                 [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]],
                                device=x.device, dtype=torch.float64)
        inner = (A[None] * (x[:, None, :] - P[None]) ** 2).sum(-1)
        return -(2.58 + (al * torch.exp(-inner)).sum(1)) / 1.94

    return [("Ackley", 1, f_ackley, False), ("Branin", 2, branin, True), ("Camel", 2, camel, False),
            ("StyTang", 2, styblinski_tang, False), ("Hartmann", 6, hartmann, True)]


def f_grad_f(f, x):
    """(f, df/dx_1, ..., df/dx_d) at x [n, d] -> [n, 1 + d] (probnum25_paper.ipynb cell 7)."""
    xs = [x[:, j].clone().requires_grad_() for j in range(x.shape[1])]
    y = f(torch.stack(xs, 1))
    grads = torch.autograd.grad(y, xs, grad_outputs=torch.ones_like(y))
    return torch.stack([y] + list(grads), 1).detach()


def paper_configs(F, device, log2n=10, iterations=5000, warm=True):
    """The paper's timing protocol (probnum25_paper.ipynb cell 15): n = 2^10 points per task, SI lattice
    alpha = 2 / DSI digital net alpha = 4, f alone (derivatives = [0]) and (f, grad f) (1 + d derivative
    tasks), fit() with the reference's defaults (Rprop lr 0.1, early stopping: improvement 5e-2 over 10
    iterations, at most 5000), store_loss_hist; time per optimisation step = fit wall time / iterations.
    With `warm`, a first untimed pass (3 iterations per config) loads every kernel before the timed pass."""
    n = 2 ** log2n
    if warm:
        paper_configs(F, device, log2n, 3, warm=False)
    out = []
    for name, d, f, bake_grad in paper_functions():
        for fam in ("lattice", "net"):
            for grad in (False, True):
                lbetas = [torch.zeros((1, d), dtype=torch.int64)]
                if grad:
                    lbetas += [e[None] for e in torch.eye(d, dtype=torch.int64)]
                T = len(lbetas)
                if fam == "lattice":
                    gp = F.FastGPLattice([F.Lattice(d, seed=7) for _ in range(T)], derivatives=lbetas, alpha=2,
                                         num_tasks=T, device=device)
                else:
                    gp = F.FastGPDigitalNetB2([F.DigitalNetB2(d, seed=7, randomize="DS") for _ in range(T)],
                                              derivatives=lbetas, alpha=4, num_tasks=T, device=device)
                xs = gp.get_x_next(n * torch.ones(T, dtype=torch.int64))
                ff = (lambda x, f=f: f(1 - 2 * torch.abs(x - 0.5))) if (fam == "lattice" and grad and bake_grad) else f
                if grad:
                    gp.add_y_next([f_grad_f(ff, xs[i])[:, i] for i in range(T)])
                else:
                    gp.add_y_next([f(xs[0])])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                data = gp.fit(iterations=iterations, verbose=0, store_loss_hist=True)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                its = max(1, int(data["iterations"]))
                col = (0 if fam == "lattice" else 2) + (1 if grad else 0)
                out.append({"benchmark": name, "d": d, "gp": "SI lattice alpha=2" if fam == "lattice" else
                            "DSI digital net alpha=4", "data": "(f, grad f)" if grad else "f", "tasks": T,
                            "n_per_task": n, "iterations": its, "s_per_step": el / its,
                            "paper_s_per_step": PAPER_S_PER_STEP[name][col],
                            "class": type(gp).__name__})
                del gp
    return out


def multitask_configs(F, device, iterations=40):
    """The reference's default multitask setting (docs/examples/multitask/fgp_lattice.ipynb cells 3-4: d = 1,
    three tasks -- low / high fidelity Ackley and a cosine sum -- at n = [2^6, 2^3, 2^8], the task kernel
    F F^T + diag(v) LEARNED, abstract_gp.py:116-139) and the same at 16x the points, each fitted `iterations`
    Rprop steps (early stopping off) through the device-resident general multitask fit (fgp_mt_fit_run) and
    through the generic autograd loop (FGP_MT_FUSED=0): time per optimisation step = fit wall time /
    iterations."""
    fs = [lambda x: f_ackley(x, c=0), lambda x: f_ackley(x), lambda x: torch.cos(2 * np.pi * x).sum(1)]
    out = []
    for scale in (1, 16):
        ns = [64 * scale, 8 * scale, 256 * scale]
        row = {"workload": "docs/examples/multitask: FastGPLattice d=1, 3 tasks, n=%s, learned task kernel" % ns,
               "iterations": iterations}
        for path in ("device", "generic"):
            old = os.environ.get("FGP_MT_FUSED")
            os.environ["FGP_MT_FUSED"] = "1" if path == "device" else "0"
            try:
                times = []
                for rep in range(2 if path == "device" else 1):       # the first device pass loads the kernels
                    gp = F.FastGPLattice(1, seed_for_seq=7, num_tasks=3, device=device)
                    xs = gp.get_x_next(n=ns)
                    gp.add_y_next([fs[i](xs[i]) for i in range(3)])
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    data = gp.fit(iterations=iterations, verbose=0, stop_crit_wait_iterations=iterations + 1,
                                  store_loss_hist=True)
                    torch.cuda.synchronize()
                    times.append((time.perf_counter() - t0) / max(1, int(data["iterations"])))
                row[path + "_s_per_step"] = min(times)
                row[path + "_final_loss"] = float(-data["loss_hist"][-1])
                if path == "device":
                    row["device_path"] = "general (fgp_mt_fit_run)" if gp._mt_general_ok() and not gp._mt_fused_ok() \
                        else ("k_mt_spec_iter" if gp._mt_fused_ok() else "generic")
            finally:
                if old is None:
                    os.environ.pop("FGP_MT_FUSED", None)
                else:
                    os.environ["FGP_MT_FUSED"] = old
        row["speedup"] = row["generic_s_per_step"] / row["device_s_per_step"]
        out.append(row)
    out += batch_multitask_configs(F, device, iterations)
    return out


def batch_multitask_configs(F, device, iterations):
    """The reference's parameter-batched multitask setting (docs/examples/batch_multitask/fgp_lattice.ipynb
    cells 4-7: d = 6, shape_batch = [2, 3, 4], 5 tasks at n = 2^[6, 5, 4, 3, 2], scale / lengthscales / noise /
    task factor / task noise batched as in cell 6) and the same at 16x the points: 24 eigen-problems per
    optimisation step through the device fit (fgp_mt_fit_run, G = 24) and through the generic autograd loop."""
    d, T, sb = 6, 5, [2, 3, 4]
    consts = torch.arange(24, device=device, dtype=torch.float64).reshape(sb)
    out = []
    for scale in (1, 16):
        ns = [scale * 2 ** k for k in range(T + 1, 1, -1)]
        row = {"workload": "docs/examples/batch_multitask: FastGPLattice d=6, 5 tasks, n=%s, shape_batch=%s, "
                           "batched scale / lengthscales / noise / task kernel" % (ns, sb), "iterations": iterations}
        for path in ("device", "generic"):
            old = os.environ.get("FGP_MT_FUSED")
            os.environ["FGP_MT_FUSED"] = "1" if path == "device" else "0"
            try:
                times = []
                for rep in range(2 if path == "device" else 1):
                    gp = F.FastGPLattice(d, seed_for_seq=7, num_tasks=T, shape_batch=sb, shape_scale=sb + [1],
                                         shape_lengthscales=sb[1:] + [d], shape_noise=sb[2:] + [1],
                                         shape_factor_task_kernel=sb + [T, T], shape_noise_task_kernel=sb[1:] + [T],
                                         device=device)
                    xs = gp.get_x_next(n=torch.tensor(ns))
                    g = torch.Generator(device=device).manual_seed(11)
                    gp.add_y_next([(consts[..., None, None] * xs[l] ** torch.arange(1, d + 1, device=device)).sum(-1)
                                   + torch.randn(sb + [xs[l].shape[0]], generator=g, device=device) / (3 + l)
                                   for l in range(T)])
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    data = gp.fit(iterations=iterations, verbose=0, stop_crit_wait_iterations=iterations + 1,
                                  store_loss_hist=True)
                    torch.cuda.synchronize()
                    times.append((time.perf_counter() - t0) / max(1, int(data["iterations"])))
                row[path + "_s_per_step"] = min(times)
                row[path + "_final_loss"] = float(-data["loss_hist"][-1])
                if path == "device":
                    row["device_path"] = "general, G=%d (fgp_mt_fit_run)" % 24 if gp._mt_general_ok() else "generic"
            finally:
                if old is None:
                    os.environ.pop("FGP_MT_FUSED", None)
                else:
                    os.environ["FGP_MT_FUSED"] = old
        row["speedup"] = row["generic_s_per_step"] / row["device_s_per_step"]
        out.append(row)
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


STAGES = ("k_fwd_rows", "k_fwd_cols", "k_bwd_rows")
SPEC_BLOCKS = 512      # k blocks per problem of the spectral iteration (csrc/fgp_nll.h kSpecBlocks)


SPEC_RING, SPEC_LDS_MAX, SPEC_MAX_DMA = 2, 80 * 1024, 6      # csrc/fgp_nll.h kSpecRing / kSpecLdsMax / kSpecMaxDma


def stage_names(variant):
    """The fit-iteration kernels of a variant, in launch order (the reduce + Rprop step aside; the fused
    spectral kernel includes it)."""
    if variant == "spectral_fused":
        return ("k_spec_tile",)
    return ("k_spec_iter",) if variant == "spectral" else STAGES


def spec_tile_geometry(n, d, G, shared=True, family=0):
    """(workgroups, problems per wave, problem groups) of the LDS-ring tile kernel k_spec_tile, or None when
    spec_geometry picks the per-wave k_spec_iter (the conditions of csrc/fgp_spectral.hip spec_geometry)."""
    main = n // 2 if family == 0 else n
    nb = min(SPEC_BLOCKS, max(1, main // 64))
    if not (shared and d <= 5 and main >= 256) or os.environ.get("FGP_SPEC_TILE", "1")[:1] == "0":
        return None
    ppw = 2 if G >= 2 else 1
    pg = (G + ppw - 1) // ppw
    pgp = 1 if pg <= 1 else (2 if pg <= 2 else 4)
    ck = 64 * (4 // pgp)
    rows = 2 ** d + G
    ok = (pg <= 4 and rows * ck * 8 * SPEC_RING <= SPEC_LDS_MAX and rows * ck <= 512 * SPEC_MAX_DMA and
          (rows * ck) % 128 == 0 and rows * ck >= 256 and nb % (4 // pgp) == 0 and main % (64 * nb) == 0)
    if ok:
        return (nb // (4 // pgp), ppw, pg)
    # problem slices (G > 8): PS = 4 PPW problems per workgroup, one k block each (64 chunks per workgroup,
    # more blocks while the grid has < 512 workgroups), snb x slices workgroups
    sppw = 4 if d <= 3 else 2
    ps = 4 * sppw
    srows = 2 ** d + ps
    nsl = (G + ps - 1) // ps
    snb = max(1, main // (64 * 64))
    while snb * nsl < 512 and snb * 2 <= max(1, main // 64):
        snb *= 2
    snb = min(snb, nb)
    if (pg > 4 and srows * 64 * 8 * SPEC_RING <= SPEC_LDS_MAX and srows * 64 <= 512 * SPEC_MAX_DMA and
            (srows * 64) % 128 == 0 and main % (64 * snb) == 0):
        return (snb * nsl, sppw, 4)
    return None


def spec_geometry(n, d, G, shared=True, family=0):
    """(k blocks, problems per wave, problem groups) of the spectral iteration (csrc/fgp_spectral.hip
    spec_geometry): the tile kernel's when it applies, else k_spec_iter's."""
    main = n // 2 if family == 0 else n
    nb = min(SPEC_BLOCKS, max(1, main // 64))
    t = spec_tile_geometry(n, d, G, shared, family)
    if t is not None:
        ps = 4 * t[1]
        sliced = (G + t[1] - 1) // t[1] > 4          # problem slices: the grid is k blocks x slices
        return (t[0] // ((G + ps - 1) // ps) if sliced else nb), t[1], t[2]
    ppw = 2 if (G >= 2 and shared and d <= 5) else 1
    if ppw == 2 and G > 8 and d <= 3:
        ppw = 4
    return nb, ppw, (G + ppw - 1) // ppw


def spec_tile_grid(n, d, G, shared=True, family=0):
    """Workgroups of the LDS-ring tile kernel k_spec_tile, or None (per-wave k_spec_iter)."""
    t = spec_tile_geometry(n, d, G, shared, family)
    return None if t is None else t[0]


def spec_fused(n, d, G):
    """fgp_fit_run runs the whole iteration (streaming + reduction + Rprop) as ONE k_spec_tile launch:
    tile geometry, per-problem parameters, G <= 8 (csrc/fgp_nll.hip fgp_fit_run)."""
    return spec_tile_grid(n, d, G) is not None and G <= 8


def r2c_active(n):
    """The lattice fit runs the half-length (R2C) or real-even (RE) kernels for n >= 2^17 unless
    FGP_R2C=0 (csrc/fgp_nll.hip to_nll)."""
    return n >= 2 ** 17 and os.environ.get("FGP_R2C", "2")[:1] != "0"


def fit_variant(n, parts_array):
    """'re' (real-even kernels: n >= 2^17 with regenerated parts, the default), 'r2c' (FGP_R2C=1, or a
    parts array) or 'full' (n < 2^17 or FGP_R2C=0) -- the choice of csrc/fgp_nll.hip to_nll."""
    if not r2c_active(n):
        return "full"
    if parts_array or os.environ.get("FGP_R2C", "2")[:1] == "1":
        return "r2c"
    return "re"


def re_row_log2():
    """Row length log2 of the real-even kernels' n/2-point transform (csrc/fgp_nll_re.hip kP2reDefault)."""
    return 11


def fit_grid(n, P, variant, d=5):
    """{stage kernel: (workgroups per fit launch, threads per workgroup)}."""
    if variant == "spectral_fused":
        return {"k_spec_tile": (spec_tile_grid(n, d, P), 256)}
    if variant == "spectral":
        if spec_tile_grid(n, d, P) is not None:       # staged tile launches (problem slices when P > 8)
            return {"k_spec_tile": (spec_tile_grid(n, d, P), 256)}
        nb, _, pg = spec_geometry(n, d, P)
        return {"k_spec_iter": ((nb * pg + 3) // 4, 256)}
    if variant == "re":     # N1 = n / (2 N2) rows of N2: N1/2 row-pair workgroups of N2/8, n/16384 column tiles
        N2 = 2 ** re_row_log2()
        N1 = n // (2 * N2)
        return {"k_fwd_rows": (P * N1 // 2, N2 // 8), "k_fwd_cols": (P * n // 16384, 256),
                "k_bwd_rows": (P * N1 // 2, N2 // 8)}
    g = P * max(1, (n // 2 if variant == "r2c" else n) // 4096)
    return {k: (g, 256) for k in STAGES}


def stage_bytes(n, d, P, parts_array, variant=None):
    """Algorithmic (compulsory) HBM bytes of one launch of each fit-iteration kernel over P lattice
    problems (complex128 intermediate `work` of L complex values; float64 Y; DESIGN.md 'Kernels'):
      full (L = n):  rows 16L write (+ 8nd parts), cols 16L + 16L + Y 8n, bwd rows 16L (+ 8nd)
      r2c (L = n/2): as full with Y 4n (Y = |y~|^2 is even, Y_k = Y_{n-k}, and the kernel reads it only
                     at each mirror pair's primary element: the n/2 values Y_k, Y_{k+n/2})
      re (L = n/4, columns [0, N2/2) of the n/2-point transform, N1 = n/(2 N2) rows of N2 = 2^11):
                     rows 16L + the Nyquist column 16 N1; cols 16L + 16L + Y 4n (the pairs (Y_2k, Y_2k+1)
                     of its frequencies) + Nyquist 16 N1 read + 4 N1 written; bwd rows 16L + 4 N1"""
    variant = variant or fit_variant(n, parts_array)
    pb = 8 * n * d if parts_array else 0
    if variant in ("spectral", "spectral_fused"):
        # one shared set of 2^d spectra of K = n/2 + 1 doubles read once per launch, Y[:K] of every
        # problem, (4 + d) partials per problem and k block written (the fused kernel's level-1 group
        # sums, reads of the partials and the parameter / history updates are < 0.1% on top)
        K = n // 2 + 1
        nb, _, _ = spec_geometry(n, d, P)
        return {stage_names(variant)[0]: 8 * K * (2 ** d) + 8 * K * P + 8 * (4 + d) * nb * P}
    if variant == "re":
        L, N1 = n // 4, n // (2 * 2 ** re_row_log2())
        return {"k_fwd_rows": (16 * L + 16 * N1) * P, "k_fwd_cols": (32 * L + 4 * n + 20 * N1) * P,
                "k_bwd_rows": (16 * L + 4 * N1) * P}
    L = n // 2 if variant == "r2c" else n
    yb = 4 * n if variant == "r2c" else 8 * n
    return {"k_fwd_rows": (16 * L + pb) * P, "k_fwd_cols": (32 * L + yb) * P, "k_bwd_rows": (16 * L + pb) * P}


def wall_clock_khz(F, device):
    import ctypes
    khz = ctypes.c_int(0)
    F._native.call("fgp_wall_clock_khz", int(device.index or 0), ctypes.byref(khz))
    return khz.value


def roofline_fit_kernels(F, shifts, iters):
    """Per-kernel timing of the batched fit iteration as launched in the step (same engine, same grid),
    two ways:
      * device clock (fgp_nll_desc.stamps): first-workgroup start to last-wave end of every launch --
        the kernel duration rocprofv3 --kernel-trace reports; this is `avg_us` and prices `achieved`;
      * HIP events recorded on torch's current stream (the stream the kernels are launched on) around
        each launch behind a spin kernel that holds the stream while the host enqueues: kernel + the
        dependent-launch gap (`avg_us_events`)."""
    shifts.reset()
    gps = shifts.gps
    n = shifts.n
    dev = torch.device(gps[0].device)
    eng = F.batch.batched_engine(gps, iters)
    eng.run(0, 2)
    torch.cuda.synchronize()
    variant = "spectral" if eng.basis is not None else fit_variant(n, eng.gen is None)
    if variant == "spectral" and spec_fused(n, eng.d, eng.G):
        variant = "spectral_fused"
    names = stage_names(variant)
    ns = len(names)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(ns + 2)] for _ in range(iters)]
    fg = fit_grid(n, eng.G, variant, eng.d)      # (workgroups, threads) per fit launch
    # room for any grid the library picks (the host mirror of its geometry, fit_grid, is checked against the
    # workgroups that actually stamped below)
    grid = max(max(g for g, _ in fg.values()), 1 << 14)
    stamps = torch.zeros((iters, ns, grid, 5), dtype=torch.int64, device=dev)   # fgp_nll_desc.stamps
    torch.cuda._sleep(int(2.4e9 * 4e-4 * iters))
    fused = variant == "spectral_fused"
    for it in range(iters):
        e = ev[it]
        e[0].record()
        if fused:     # the step's own launch: one kernel per iteration (fgp_fit_run), stamped
            eng._nll.stamps = stamps[it, 0].data_ptr()
            eng.run(it, 1)
            e[1].record()
            e[2].record()
            continue
        for k in range(ns):
            eng._nll.stamps = stamps[it, k].data_ptr()
            eng.stage(k)
            e[k + 1].record()
        eng._nll.stamps = None
        eng.fit_step(it)
        e[ns + 1].record()
    eng._nll.stamps = None
    torch.cuda.synchronize()
    eng._nll.stamps = None
    khz = wall_clock_khz(F, dev)
    st = stamps.cpu()
    dur = []
    for k, name in enumerate(names):    # records [workgroup][start, wave ends...] of this launch's grid
        g, thr = fg[name]
        stamped = int((st[0, k, :, 0] > 0).sum())
        if stamped != g:                 # the library chose another geometry than the host mirror (small n)
            g = stamped
            fg[name] = (g, thr)
        sk = st[:, k, :g, :1 + thr // 64]
        assert g > 0 and bool((sk > 0).all()), "a fit launch did not write its device-clock stamps"
        dur.append((sk[..., 1:].amax((1, 2)) - sk[..., 0].amin(1)).double() * (1e3 / khz))
    dur_us = torch.stack(dur, 1)     # [iters, ns]
    us_ev = {name: 1e3 * sum(e[k].elapsed_time(e[k + 1]) for e in ev) / iters for k, name in enumerate(names)}
    if fused:
        # the per-launch events above include one counter reset per fgp_fit_run call; the step makes ONE
        # call for all its iterations -- time that (events around eng.run(0, iters)) for the iteration
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 2e-4))
        e0.record()
        eng.run(0, iters)
        e1.record()
        torch.cuda.synchronize()
        us_ev = {names[0]: 1e3 * e0.elapsed_time(e1) / iters}
        # the same call replayed from a hipGraph, as the timed step runs it (a replayed launch skips the eager
        # enqueue's per-packet work): HIP events around the replays, per iteration
        us_ev[names[0] + "@graph"] = graph_fit_us(eng, iters)
    us = {name: float(dur_us[:, k].mean()) for k, name in enumerate(names)}
    if not fused:
        us_ev["k_fit_reduce_step"] = 1e3 * sum(e[ns].elapsed_time(e[ns + 1]) for e in ev) / iters
        us["k_fit_reduce_step"] = us_ev["k_fit_reduce_step"]
    t_iter = sum(v for k, v in us_ev.items() if not k.endswith("@graph")) / 1e6
    return n, variant, us, us_ev, t_iter, khz


def graph_fit_us(eng, iters, reps=5):
    """Per-iteration time of eng.run(0, iters) (fgp_fit_run: one k_spec_tile per iteration + the final step)
    captured once into a hipGraph and replayed `reps` times between two HIP events; None when the capture fails."""
    try:
        cur = torch.cuda.current_stream()
        s = torch.cuda.Stream()
        s.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                eng.run(0, iters)
        cur.wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return 1e3 * e0.elapsed_time(e1) / (reps * iters)
    except Exception:                   # capture not possible here
        _clear_capture_error()
        return None


ROOT = os.path.dirname(os.path.abspath(__file__))
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06x_pmc_fit_kernels.json")
PMC_SQ_SUMMARY = os.path.join(ROOT, "profiles", "r06x_pmc_sq_fit_kernels.json")
ROCPROF_GRID_STATS = os.path.join(ROOT, "profiles", "r06x_bench_timed_region_stats.txt")
# the read floor of the spectral iteration's footprint: tools/stream_microbench.hip over the same 168 MB,
# re-read back to back, 24.0-24.3 us per pass (7.0 TB/s; profiles/r03v_stream_and_stamps.jsonl)
STREAM_FLOOR_US = 24.0
# FP64 VALU lane-operations per second: 256 CUs x 4 SIMDs x 16 FP64 lanes per clock x 2.4 GHz = 3.93e13
# (FP64 vector at half the FP32 vector rate of MI355X_MICROARCH.md, 157.3 TFLOP/s; 78.6 TFLOP/s FMA)
FP64_LANE_OPS_PEAK = 256 * 4 * 16 * 2.4e9
CPU_FIDELITY = os.path.join(ROOT, "profiles", "r02_cpu_fidelity.json")
# the prediction kernels (tools/predict_kernels.py: C4's batched post_mean / post_var, C5 per-output's post_mean):
# rocprofv3 kernel-trace summary and SQ counter pass
ROCPROF_PREDICT_STATS = os.path.join(ROOT, "profiles", "r06x_predict_kernel_grid_stats.txt")
PMC_SQ_PREDICT = os.path.join(ROOT, "profiles", "r06x_pmc_sq_predict.json")


def pmc_traffic(kernel, grid):
    """HBM bytes per launch of `kernel` at `grid` threads from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py over FETCH_SIZE / WRITE_SIZE passes of tools/fit_kernels.py, same kernels
    and grid; FETCH_SIZE x2 gfx950 correction), or None when absent."""
    try:
        summ = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None
    for k, v in summ.items():
        name, _, g = k.partition("|grid=")
        if name.split("<")[0].split("::")[-1] == kernel and g == str(grid) and "traffic_bytes" in v:
            return v["traffic_bytes"]
    return None


def _kernel_match(name, kernel):
    """`kernel` is a base name ("k_spec_tile": any template instance) or a full instance ("k_post_mean<0, 5, 1, 4>")."""
    full = name.split("::")[-1] if "<" not in name else name[name.index("k_"):] if "k_" in name else name
    if "<" in kernel:
        return full.replace(" ", "") == kernel.replace(" ", "")
    return name.split("<")[0].split("::")[-1] == kernel


def pmc_valu_insts(kernel, grid, path=None):
    """VALU wave-instructions per launch (SQ_INSTS_VALU) of `kernel` at `grid` threads from the committed
    SQ counter pass (tools/pmc_sq_summary.py over tools/fit_kernels.py; `path`: another summary, e.g. the
    prediction kernels' over tools/predict_kernels.py), or None when absent."""
    try:
        summ = json.load(open(path or PMC_SQ_SUMMARY))
    except (OSError, ValueError):
        return None
    for k, v in summ.items():
        name, _, g = k.partition("|grid=")
        if _kernel_match(name, kernel) and (grid is None or g == str(grid)) and "SQ_INSTS_VALU" in v:
            return v["SQ_INSTS_VALU"]
    return None


def rocprof_avg_us(kernel, grid, path=None):
    """Average duration of `kernel` at `grid` threads in the committed rocprofv3 --kernel-trace summary
    of this bench command (tools/kstats_grid.py over `rocprofv3 --kernel-trace --stats -- python3
    bench.py`; `path`: another summary), or None when absent."""
    try:
        lines = open(path or ROCPROF_GRID_STATS).read().splitlines()[1:]
    except OSError:
        return None
    for ln in lines:
        f = ln.split()
        if len(f) < 6:
            continue
        name = " ".join(f[:-5])
        if _kernel_match(name, kernel) and (grid is None or f[-5] == str(grid)):
            return float(f[-3])
    return None


def post_mean_ops_per_pair(d, nb):
    """FP64 VALU instructions per (test point, training point, output) of k_post_mean's folded-B4 loop
    (csrc/fgp_predict.hip; lattice, alpha = 2), read off its gfx950 ISA: per dimension v_add_f64 (x_t - z_i) and
    v_fma_f64 (u = t^2 - |t|) shared by the kernel's nb outputs, then per output v_fma_f64 (u^2 + c') and v_mul_f64
    into the product (less the first dimension's product by 1.0), and one v_fmac_f64 with the coefficient:
    (2 d + 2 d nb) / nb -- 4 d for one output."""
    return (2.0 * d + 2.0 * d * nb) / nb


def roofline_post_mean(kernel, grid, pairs, d, nb, stats=None, sq=None, live_ms=None, launches=1):
    """FP64-VALU roofline of a posterior-mean launch (abstract_gp.py:352-380; matrix-free cross-kernel
    contraction): `pairs` (test point, training point, output) triples per launch x post_mean_ops_per_pair
    lane-operations over the rocprofv3 average duration, against the FP64 VALU issue peak; beside it the
    measured SQ_INSTS_VALU x 64 lanes over the same duration (every VALU instruction, address and loop
    arithmetic included)."""
    us = rocprof_avg_us(kernel, grid, stats)
    ops = post_mean_ops_per_pair(d, nb)
    out = {"bound": "fp64 valu", "kernel": kernel, "pairs_per_launch": pairs, "ops_per_pair": ops,
           "op_model": "per dimension v_add_f64 + v_fma_f64 shared by %d output(s), v_fma_f64 + v_mul_f64 per output, "
                       "one v_fmac_f64 per output (gfx950 ISA of the folded-B4 loop)" % nb,
           "peak": FP64_LANE_OPS_PEAK, "unit": "FP64 lane-ops/s", "launches_per_step": launches,
           "avg_us_source": "rocprofv3 --kernel-trace average, %s" % os.path.relpath(stats or ROCPROF_GRID_STATS, ROOT)}
    if us is None:
        return out
    ach = pairs * ops / (us * 1e-6)
    out.update({"avg_us": us, "achieved": ach, "frac": ach / FP64_LANE_OPS_PEAK})
    vi = pmc_valu_insts(kernel, grid, sq)
    if vi is not None:
        out["valu"] = {"insts_per_launch": vi, "frac": vi * 64 / (us * 1e-6) / FP64_LANE_OPS_PEAK,
                       "source": os.path.relpath(sq or PMC_SQ_SUMMARY, ROOT) + " (SQ_INSTS_VALU)"}
    if live_ms is not None:
        out["phase_ms_live"] = live_ms
    return out


SECONDARY_STATS = os.path.join(ROOT, "profiles", "r06k_secondary_stats.json")
FP64_MFMA_PEAK_FLOPS = 78.6e12       # MI355X FP64 matrix peak (spec; = the FP64 vector FMA rate)


def secondary_rooflines(case, n, d, outputs, n_mean, fit_iters):
    """Rooflines of a secondary line's kernels, priced on the committed rocprofv3 trace + PMC passes
    of the same steps (tools/secondary_profile.sh -> tools/secondary_kernels.py, profiles/r06k_secondary_stats.json;
    durations: the kernel trace's per-launch averages; traffic: FETCH_SIZE x2 (gfx950) + WRITE_SIZE per launch).
    Returns [primary, others...] (primary = the line's longest kernel per step) or []."""
    try:
        st = json.load(open(SECONDARY_STATS))
    except (OSError, ValueError):
        return []
    tr = st["trace"].get(case)
    if not tr:
        return []
    src = os.path.relpath(SECONDARY_STATS, ROOT)

    def find(prefix):
        for k, v in tr.items():
            if k.startswith(prefix):
                return k, v
        return None, None

    def counters(k):
        f = st.get("fetch_kb", {}).get(case, {}).get(k)
        w = st.get("write_kb", {}).get(case, {}).get(k)
        q = st.get("sq_insts_valu", {}).get(case, {}).get(k)
        return (None if f is None or w is None else 2.0 * f * 1024 + w * 1024), q

    def hbm(k, v, alg, what):
        traffic, q = counters(k)
        ach = alg / (v["avg_us"] * 1e-6) / 1e9
        r = {"bound": "hbm", "kernel": k.split("|")[0], "grid_threads": int(k.split("=")[-1]), "algorithmic_bytes": alg,
             "bytes_model": what, "avg_us": v["avg_us"], "launches_per_step": v["launches_per_step"],
             "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
             "source": src}
        if q is not None:
            r["valu_frac"] = q * 64 / (v["avg_us"] * 1e-6) / FP64_LANE_OPS_PEAK
        return r

    K = n // 2 + 1 if case != "C3" else n
    out = []
    if case in ("C2", "C3"):
        k, v = find("k_spec_persist")
        if k is not None:
            traffic, q = counters(k)
            ach = q * 64 / (v["avg_us"] * 1e-6) if q is not None else None
            lds = 8 * K * (2 ** d + 1)        # the spectra + Y, LDS-resident, read once per iteration
            out.append({"bound": "latency (one grid barrier + reduction + Rprop step per iteration)", "kernel": k.split("|")[0],
                        "grid_threads": int(k.split("=")[-1]), "avg_us": v["avg_us"], "iterations": fit_iters + 1,
                        "iteration_us": v["avg_us"] / (fit_iters + 1), "achieved": ach, "peak": FP64_LANE_OPS_PEAK,
                        "unit": "FP64 lane-ops/s (SQ_INSTS_VALU x 64)", "frac": None if ach is None else ach / FP64_LANE_OPS_PEAK,
                        "lds_bytes_per_iteration": lds, "hbm_traffic_per_launch": traffic,
                        "note": "the whole 51-iteration fit in one launch (fgp_fit_persist): spectra + Y stay in LDS, so "
                                "neither HBM nor VALU bounds the iteration; its time is the in-kernel barrier chain",
                        "source": src})
    if case in ("C5", "C5 mixed"):
        k, v = find("Cijk_")
        if k is not None:
            flops = 2.0 * n_mean * n * outputs / v["launches_per_step"]
            ach = flops / (v["avg_us"] * 1e-6)
            out.append({"bound": "mfma (fp64)", "kernel": "library DGEMM (post_mean: kernel rows x coefficients)",
                        "kernel_symbol": k.split("|")[0][:80], "flops_per_launch": flops,
                        "flops_model": "2 N n B over its launches per step", "avg_us": v["avg_us"],
                        "launches_per_step": v["launches_per_step"], "achieved": ach / 1e12, "peak": FP64_MFMA_PEAK_FLOPS / 1e12,
                        "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_FLOPS, "traffic": counters(k)[0], "source": src})
        k, v = find("k_inv_cols_c2r")
        if k is not None:
            out.append(hbm(k, v, 32.0 * (n // 2) * outputs, "coefficients, column pass: 16 (n/2) B read + 16 (n/2) B written"))
        k, v = find("k_inv_rows_c2r")
        if k is not None:
            out.append(hbm(k, v, (16.0 * (n // 2) + 8.0 * n) * outputs, "coefficients, row pass: 16 (n/2) B read + 8 n B written"))
        k, v = find("k_spec_persist")
        if k is not None:
            traffic, q = counters(k)
            out.append({"bound": "latency (single-launch fit)", "kernel": k.split("|")[0], "avg_us": v["avg_us"],
                        "iteration_us": v["avg_us"] / (fit_iters + 1), "frac": None if q is None else
                        q * 64 / (v["avg_us"] * 1e-6) / FP64_LANE_OPS_PEAK, "unit": "FP64 VALU fraction", "source": src})
    if case == "C5 per-output":
        k, v = find("k_spec_tile")
        if k is not None:
            out.append(hbm(k, v, 8.0 * K * (2 ** d) + 8.0 * K * outputs,
                           "one fit iteration of %d problems sharing the spectra: 2^d spectra + Y of every problem, "
                           "8 K bytes each (K = n/2 + 1)" % outputs))
        k, v = find("k_spec_post_var")
        if k is not None:
            traffic, q = counters(k)
            if q is not None:
                ach = q * 64 / (v["avg_us"] * 1e-6)
                out.append({"bound": "fp64 valu", "kernel": k.split("|")[0], "avg_us": v["avg_us"],
                            "launches_per_step": v["launches_per_step"], "achieved": ach, "peak": FP64_LANE_OPS_PEAK,
                            "unit": "FP64 lane-ops/s (SQ_INSTS_VALU x 64)", "frac": ach / FP64_LANE_OPS_PEAK,
                            "traffic": traffic, "note": "post_var of the %d problems by linearity of the test points' row "
                            "spectra: per (problem, test point, frequency) the 2^d-term polynomial" % outputs,
                            "source": src})
    out.sort(key=lambda r: -(r.get("avg_us", 0) * r.get("launches_per_step", 1)))
    return out


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


def _clear_capture_error():
    """After an invalidated capture the HIP error is reported by the next launch: take it here (a throwaway
    op whose error is swallowed) so the eager fallback runs clean."""
    for _ in range(3):
        try:
            torch.zeros(1, device="cuda").add_(1)
            torch.cuda.synchronize()
            return
        except Exception:
            continue


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
