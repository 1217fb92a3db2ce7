"""Kernel trace helper: a few eager C5 steps (bench.MultiOutputGP + bench.step_single, 512 outputs at n = 2^18, d = 3)
of the shared, per-output or fp32 variant; run under rocprofv3 --kernel-trace."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fastgaussianprocesses_amd as F  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--variant", default="shared", choices=["shared", "per_output", "fp32"])
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
dev = "cuda:0"
sg = bench.MultiOutputGP(F, 18, 3, 512, dev, torch.float32 if a.variant == "fp32" else torch.float64,
                         per_output=a.variant == "per_output")
g = torch.Generator().manual_seed(17)
xm = torch.rand((256, 3), generator=g).to(dev)
xv = torch.rand((8, 3), generator=g).to(dev)
args = argparse.Namespace(fit_iters=50)
for r in range(a.reps):
    bench.step_single(sg, args, xm, xv)
    torch.cuda.synchronize()
print("done", flush=True)
