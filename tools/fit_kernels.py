"""Launch only the fit-iteration kernels of the bench workload (for rocprofv3 --pmc passes).

  python tools/fit_kernels.py [--log2n 20] [--d 5] [--shifts 8] [--iters 5] [--parts-array]

Builds the same batched engine as bench.py's step (bench.Shifts + fastgaussianprocesses_amd.batch)
and runs `--iters` iterations as the step launches them (spectral path: one fused k_spec_tile per
iteration; transform path: stage 0/1/2 + fit step), so a counter pass sees a few dispatches at the
bench's grid.
"""
import argparse
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
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--parts-array", action="store_true")
    a = p.parse_args()
    if a.parts_array:
        os.environ["FGP_PARTS_GEN"] = "0"
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    shifts = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(a.shifts)], dev)
    shifts.reset()
    eng = F.batch.batched_engine(shifts.gps, a.iters)
    if eng.basis is not None:       # spectral path: the step's own launches (one fused kernel per iteration)
        eng.run(0, a.iters)
    else:
        for it in range(a.iters):
            for k in range(3):
                eng.stage(k)
            eng.fit_step(it)
    torch.cuda.synchronize()
    print("ran %d fit iterations over %d problems, n=2^%d, d=%d, parts=%s" %
          (a.iters, a.shifts, a.log2n, a.d, "array" if eng.gen is None else "regenerated"))


if __name__ == "__main__":
    main()
