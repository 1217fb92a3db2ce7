"""Fit-iteration time of the batched real-even fit across sizes (8 lattice GPs, d = 5).

  python tools/exp_size_sweep.py [--mmin 16] [--mmax 22] [--iters 20]

For each n = 2^m: one fgp_fit_run of `iters` iterations over 8 problems (the bench's engine), timed with
HIP events behind a sleep kernel that holds the stream.  Prints one JSON line per size: microseconds per
iteration, points per second (8 n per iteration) and the iteration's compulsory bytes (20 n per problem)
per second.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mmin", type=int, default=16)
    p.add_argument("--mmax", type=int, default=22)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    for m in range(a.mmin, a.mmax + 1):
        n = 2 ** m
        sh = bench.Shifts(F, a.d, n, [1000 + s for s in range(8)], dev)
        sh.reset()
        eng = F.batch.batched_engine(sh.gps, a.iters)
        raw0 = eng.raw.clone()
        eng.run(0, a.iters)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.raw.copy_(raw0)
        torch.cuda._sleep(int(2.4e9 * 5e-4))
        e0.record()
        eng.run(0, a.iters)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps({"log2n": m, "problems": 8, "d": a.d, "us_per_iter": us, "points_per_s": 8 * n / (us * 1e-6),
                          "compulsory_GBps": 8 * 20 * n / (us * 1e-6) / 1e9}), flush=True)
        del eng, sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
