"""Launch only the C5 per-output fit (512 eigen-problems sharing one set of spectra: k_spec_iter with
4 problems per wave) for rocprofv3 --pmc passes.   python tools/spec_many.py [--iters 5] [--outputs 512]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--outputs", type=int, default=512)
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sg = bench.MultiOutputGP(F, 18, 3, a.outputs, dev, per_output=True)
    sg.reset()
    sg.gp.fit(iterations=a.iters, stop_crit_wait_iterations=a.iters + 1, verbose=0)
    torch.cuda.synchronize()
    print("ran %d fit iterations of %d per-output problems" % (a.iters, a.outputs))


if __name__ == "__main__":
    main()
