"""(Historical: the FGP_SPEC_EXP_NOCOMPUTE switch these runs used was removed from the product kernel
after the round-3 measurements; its 'stream' rows need a build of commit e26f9e6.)
Spectral fit path timing on one GPU (C4 shape by default: 8 shifted lattice GPs, n = 2^20, d = 5):
basis build, the iteration kernel alone (stage launches) and the fused fit loop per iteration, for the
tile kernel, the per-wave kernel (FGP_SPEC_TILE=0) and the transform path (FGP_FIT_PATH=transform).
Prints one JSON line per variant.  HIP events on torch's current stream.

    python tools/exp_spec.py [--log2n 20] [--d 5] [--shifts 8] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def ev_time(fn, reps=1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2e6))
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--d", type=int, default=5)
    ap.add_argument("--shifts", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    n = 2 ** args.log2n
    sh = bench.Shifts(F, args.d, n, bench.shard_seeds(0, 1, args.shifts), dev)
    sh.reset()
    b = sh.batch
    out = {"ytilde_ms": ev_time(lambda: (b._st.pop("yt", None), b._st.pop("ysq", None), b.ysq()), 3)}
    out["basis_ms"] = ev_time(lambda: (b._st.pop("basis", None), b.basis()), 3)
    bas = b.basis()
    out["basis_MB"] = bas.numel() * 8 / 1e6
    out["basis_sum_us"] = 1e3 * ev_time(lambda: bas.sum(), 10)          # a plain streaming read, calibration
    out["basis_sum_GBps"] = bas.numel() * 8 / (out["basis_sum_us"] * 1e-6) / 1e9
    print(json.dumps(out), flush=True)
    # one problem alone on the same spectra (G = 1): memory-bound if it takes as long as G = 8
    os.environ.update({"FGP_FIT_PATH": "spectral", "FGP_SPEC_TILE": "1"})
    from fastgaussianprocesses_amd.fit_engine import FusedMLL, mll_constant
    ysq1 = b.ysq()[:1].contiguous()
    raw = b.raw()
    os.environ["FGP_SPEC_EXP_NOCOMPUTE"] = "1"
    e8 = FusedMLL(0, None, b.ysq()[:8].contiguous(), raw[:8, 0], raw[:8, 1:1 + args.d], raw[:8, -1], 1.0,
                  mll_constant(1, n), max_iters=4, per_problem=True, basis=bas)
    print(json.dumps({"variant": "tile stage kernel, G=8, streaming only (no terms)",
                      "us": 1e3 * ev_time(lambda: e8.stage(0), 20)}), flush=True)
    os.environ.pop("FGP_SPEC_EXP_NOCOMPUTE")
    for G in (1, 2, 4, 8):
        e1 = FusedMLL(0, None, b.ysq()[:G].contiguous(), raw[:G, 0], raw[:G, 1:1 + args.d], raw[:G, -1], 1.0,
                      mll_constant(1, n), max_iters=4, per_problem=True, basis=bas)
        t1 = ev_time(lambda: e1.stage(0), 20)
        print(json.dumps({"variant": "tile stage kernel, G=%d" % G, "us": 1e3 * t1}), flush=True)
    for name, env in (("tile", {"FGP_FIT_PATH": "spectral", "FGP_SPEC_TILE": "1"}),
                      ("per-wave", {"FGP_FIT_PATH": "spectral", "FGP_SPEC_TILE": "0"}),
                      ("transform", {"FGP_FIT_PATH": "transform"})):
        os.environ.update(env)
        sh.reset()
        eng = F.batch.batched_engine(sh.gps, args.iters)
        eng.run(0, 2)
        torch.cuda.synchronize()
        it = args.iters
        t_run = ev_time(lambda: eng.run(0, it)) / it
        nst = 1 if eng.basis is not None else 3

        def stages():
            for k in range(nst):
                eng.stage(k)
        t_stage = ev_time(stages, 20)
        t_step = ev_time(lambda: eng.fit_step(0), 20)
        print(json.dumps({"variant": name, "fit_run_us_per_iter": 1e3 * t_run, "stage_kernels_us": 1e3 * t_stage,
                          "fit_step_us": 1e3 * t_step, "basis": eng.basis is not None}), flush=True)
    os.environ.pop("FGP_SPEC_TILE", None)
    os.environ.pop("FGP_FIT_PATH", None)


if __name__ == "__main__":
    main()
