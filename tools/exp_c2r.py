"""Timing of the real-input forward / real-output inverse transforms, half length vs full length.

  python tools/exp_c2r.py [--log2n 18] [--batch 512] [--reps 5]

HIP events behind a sleep kernel; prints one JSON line per transform: microseconds per call (half / full
length) and the bytes each moves per call (half: 40n / 40n per row; full: 56n / 56n per row).
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
    p.add_argument("--log2n", type=int, default=18)
    p.add_argument("--batch", type=int, default=512)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    n, B = 2 ** a.log2n, a.batch
    x = torch.randn((B, n), device=dev)
    X = F.ops.fftbr_raw(x)
    f = torch.rand((1, n), device=dev).to(torch.complex128)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 1e-3))
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    out = {}
    for mode in ("2", "0"):
        os.environ["FGP_R2C"] = mode
        tag = "half" if mode == "2" else "full"
        out["fwd_" + tag + "_us"] = timed(lambda: F.ops.fftbr_raw(x))
        out["inv_mul_" + tag + "_us"] = timed(lambda: F.ops.inverse_mul(F.ops.LATTICE, X, f, real_out=True))
    out["rows"] = B
    out["log2n"] = a.log2n
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
