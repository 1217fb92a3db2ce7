"""One C2 / C3 step (bench.SingleGP, n = 2^16, d = 3, 50 Rprop iterations + post_mean 256 + post_var 8) repeated
eagerly, with the phase boundaries printed as device-event times -- run under rocprofv3 --kernel-trace to see
which kernels make up ytilde+fit."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fastgaussianprocesses_amd as F  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--family", default="lattice")
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
dev = "cuda:0"
sg = bench.SingleGP(F, a.family, 16, 3, dev)
g = torch.Generator().manual_seed(17)
xm = torch.rand((256, 3), generator=g).to(dev)
xv = torch.rand((8, 3), generator=g).to(dev)
for r in range(a.reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    sg.reset()
    ev[0].record()
    sg.gp.fit(iterations=50, stop_crit_wait_iterations=51, verbose=0)
    ev[1].record()
    with torch.no_grad():
        sg.gp.coeffs
    ev[2].record()
    sg.gp.post_mean(xm)
    sg.gp.post_var(xv)
    ev[3].record()
    torch.cuda.synchronize()
    print("rep %d: ytilde+fit %.3f ms, coeffs %.3f ms, predict %.3f ms"
          % (r, ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])), flush=True)
