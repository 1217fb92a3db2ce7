"""Experiment: can one problem group's VALU-bound row kernel overlap another group's column kernel?

  python tools/exp_overlap.py [--log2n 20] [--d 5] [--shifts 8] [--reps 40]

Splits the bench's 8 problems into two groups (FusedMLL._group_descs) and times, per pair of stages
(a, b): group A's stage a and group B's stage b back to back on one stream (serial) against the two on
two streams started together (concurrent).  Prints one JSON line per pair.
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
    p.add_argument("--reps", type=int, default=40)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    from fastgaussianprocesses_amd import _native as N
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(a.shifts)], dev)
    sh.reset()
    eng = F.batch.batched_engine(sh.gps, 4)
    (na, _, _), (nb, _, _) = eng._group_descs(2)[:2]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    for k in range(3):
        N.call("fgp_nll_stage", na, k, cur.cuda_stream)
        N.call("fgp_nll_stage", nb, k, cur.cuda_stream)
    torch.cuda.synchronize()

    def timed(fn):
        """GPU time per call: the calls are enqueued behind a sleep kernel that holds the stream, so
        host launch overhead is not measured."""
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 8e-5 * a.reps))
        e0.record(cur)
        for _ in range(a.reps):
            fn()
        e1.record(cur)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    names = {0: "fwd_rows", 1: "fwd_cols", 2: "bwd_rows"}
    for sa, sb in ((0, 1), (2, 1), (0, 2), (0, 0), (1, 1)):
        def serial():
            N.call("fgp_nll_stage", na, sa, cur.cuda_stream)
            N.call("fgp_nll_stage", nb, sb, cur.cuda_stream)

        def concurrent():
            ev = torch.cuda.Event()
            ev.record(cur)
            s1.wait_event(ev)
            s2.wait_event(ev)
            N.call("fgp_nll_stage", na, sa, s1.cuda_stream)
            N.call("fgp_nll_stage", nb, sb, s2.cuda_stream)
            e1, e2 = torch.cuda.Event(), torch.cuda.Event()
            e1.record(s1)
            e2.record(s2)
            cur.wait_event(e1)
            cur.wait_event(e2)

        def alone_a():
            N.call("fgp_nll_stage", na, sa, cur.cuda_stream)

        def alone_b():
            N.call("fgp_nll_stage", nb, sb, cur.cuda_stream)

        r = dict(a=names[sa], b=names[sb], alone_a_us=timed(alone_a), alone_b_us=timed(alone_b),
                 serial_us=timed(serial), concurrent_us=timed(concurrent))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
