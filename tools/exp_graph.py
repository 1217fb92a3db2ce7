"""Experiment: the fused fit loop (fgp_fit_run, 3 launches per iteration) replayed from a HIP graph
against eager enqueueing, on the bench's 8 problems at n = 2^20, d = 5.

  python tools/exp_graph.py [--iters 50] [--reps 5]

Prints one JSON line: microseconds per fit iteration, eager and graph.
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
    p.add_argument("--shifts", type=int, default=8)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(a.shifts)], dev)
    sh.reset()
    eng = F.batch.batched_engine(sh.gps, a.iters)
    raw0 = eng.raw.clone()
    eng.run(0, a.iters)
    torch.cuda.synchronize()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 2e-3))
        e0.record()
        for _ in range(a.reps):
            eng.raw.copy_(raw0)
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (a.reps * a.iters)

    out = {"eager_us_per_iter": timed(lambda: eng.run(0, a.iters))}
    hist_eager = eng.loss_hist[:a.iters].clone()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eng.raw.copy_(raw0)
        eng.run(0, a.iters)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            eng.run(0, a.iters)
        out["graph_us_per_iter"] = timed(g.replay)
        out["graph_equal_eager"] = bool(torch.equal(eng.loss_hist[:a.iters], hist_eager))
    except Exception as e:  # noqa: BLE001
        out["graph_error"] = repr(e)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
