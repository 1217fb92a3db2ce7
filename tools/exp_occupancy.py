"""Experiment: are the real-even fit kernels limited by a CU-wide throughput or by latency?

  python tools/exp_occupancy.py [--log2n 20] [--d 5] [--reps 20]

Times each fit stage (fgp_nll_stage, HIP events behind a sleep kernel that holds the stream) for P = 1, 2,
4, 8 problems: the row kernels launch 128 workgroups per problem at n = 2^20 (P = 2: one per CU; P = 8: four
per CU).  If the time grows ~linearly from P = 2 to P = 8, co-resident workgroups do not overlap (a
CU-wide throughput limit); if it stays flat, the kernel is latency-bound at one workgroup per CU.
Prints one JSON line per P.
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
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(8)], dev)
    for P in (1, 2, 4, 8):
        sh.reset()
        eng = F.batch.batched_engine(sh.gps[:P], 4)
        for k in range(3):
            eng.stage(k)
        torch.cuda.synchronize()
        out = {"P": P}
        for k, name in enumerate(("fwd_rows", "fwd_cols", "bwd_rows")):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(int(2.4e9 * 6e-5 * a.reps))
            e0.record()
            for _ in range(a.reps):
                eng.stage(k)
            e1.record()
            torch.cuda.synchronize()
            out[name + "_us"] = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
