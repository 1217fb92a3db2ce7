"""The secondary bench lines' steps (bench.secondary_configs: C2, C3, C5 shared fp64, C5 per-output, C5 fp32 data), each
run eagerly `--steps` times between two device-clock marker launches (k_clock_stamp), for rocprofv3 kernel traces and
--pmc passes: tools/secondary_stats.py splits the trace at the markers and reports per case the kernels of one step
(launches, average duration, grid) -- the durations bench.py prices each secondary line's roofline on.

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o p -- python3 tools/secondary_kernels.py
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)

CASES = ("C2", "C3", "C5", "C5 per-output", "C5 mixed")


def make(F, bench, name, dev, outputs):
    if name == "C2":
        return bench.SingleGP(F, "lattice", 16, 3, dev), 3
    if name == "C3":
        return bench.SingleGP(F, "net", 16, 3, dev), 3
    if name == "C5":
        return bench.MultiOutputGP(F, 18, 3, outputs, dev), 3
    if name == "C5 per-output":
        return bench.MultiOutputGP(F, 18, 3, outputs, dev, per_output=True), 3
    return bench.MultiOutputGP(F, 18, 3, outputs, dev, torch.float32), 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--outputs", type=int, default=512)
    ap.add_argument("--cases", default=",".join(CASES))
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    marks = torch.zeros(2, dtype=torch.int64, device=dev)
    stamp = lambda: F._native.call("fgp_clock_stamp", marks.data_ptr(), torch.cuda.current_stream().cuda_stream)
    bargs = argparse.Namespace(fit_iters=50, n_mean=256, n_var=8)
    for name in args.cases.split(","):
        sg, d = make(F, bench, name, dev, args.outputs)
        g = torch.Generator().manual_seed(17)
        xm = torch.rand((bargs.n_mean, d), generator=g).to(dev)
        xv = torch.rand((bargs.n_var, d), generator=g).to(dev)
        for _ in range(2):
            bench.step_single(sg, bargs, xm, xv)
        torch.cuda.synchronize()
        stamp()                                   # marker: the case's steps follow
        for _ in range(args.steps):
            bench.step_single(sg, bargs, xm, xv)
        stamp()
        torch.cuda.synchronize()
        print("case %s: %d steps" % (name, args.steps), flush=True)
        del sg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
