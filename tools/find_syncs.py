"""Diagnostic: list the host synchronisations inside one bench step (torch.cuda.set_sync_debug_mode).

  python tools/find_syncs.py [--log2n 20] [--d 5]

Runs a warm-up step, then one step of bench.step_batched with the sync debug mode on "warn" and prints
each synchronising call site (the innermost frames under this repository).
"""
import argparse
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(8)], dev)
    g = torch.Generator().manual_seed(3)
    xm = torch.rand((256, a.d), generator=g).to(dev)
    xv = torch.rand((8, a.d), generator=g).to(dev)

    class Args:
        fit_iters = 50

    bench.step_batched(sh, Args, xm, xv)
    torch.cuda.synchronize()
    sites = []

    def hook(message, category, filename, lineno, file=None, line=None):
        st = [f for f in traceback.extract_stack() if ROOT in f.filename and "find_syncs" not in f.filename]
        sites.append((str(message)[:80], [(os.path.relpath(f.filename, ROOT), f.lineno, f.line) for f in st[-3:]]))

    warnings.showwarning = hook
    torch.cuda.set_sync_debug_mode("warn")
    bench.step_batched(sh, Args, xm, xv)
    torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    print("%d synchronising calls in one step" % len(sites))
    for msg, st in sites:
        print(msg)
        for f, ln, src in st:
            print("    %s:%d  %s" % (f, ln, src))


if __name__ == "__main__":
    main()
