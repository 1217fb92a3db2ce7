"""Per-stage device-clock times of the batched fit iteration (bench workload, bench.roofline_fit_kernels)
and the wall time of `--iters` fused iterations (FusedMLL.run), for A/B experiments:

    FGP_LIB_PATH=... python tools/stage_times.py [--log2n 20] [--d 5] [--shifts 8] [--iters 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    p.add_argument("--shifts", type=int, default=8)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--tag", default="")
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(a.shifts)], dev)
    n, parts_array, us, us_ev, t_iter, khz = bench.roofline_fit_kernels(F, sh, a.iters)
    sh.reset()
    eng = F.batch.batched_engine(sh.gps, a.iters)
    eng.run(0, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(0, a.iters)
    torch.cuda.synchronize()
    run_us = (time.perf_counter() - t0) / a.iters * 1e6
    print(json.dumps({"tag": a.tag, "lib": os.environ.get("FGP_LIB_PATH", "default"),
                      "stage_us": {k: round(v, 2) for k, v in us.items()},
                      "run_us_per_iter": round(run_us, 2)}))


if __name__ == "__main__":
    main()
