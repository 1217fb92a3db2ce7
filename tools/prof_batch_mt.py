"""Where the time of a parameter-batched multitask fit goes (bench.batch_multitask_configs, scale 1): wall time
of the engine build, of one eng.run over the whole fit, and of gp.fit; run under rocprofv3 --kernel-trace --stats
for the device side."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fastgaussianprocesses_amd as F  # noqa: E402
from fastgaussianprocesses_amd.multitask import MtGeneralEngine  # noqa: E402

torch.set_default_dtype(torch.float64)
dev = "cuda:0"
d, T, sb = 6, 5, [2, 3, 4]
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 1
its = 40
consts = torch.arange(24, device=dev, dtype=torch.float64).reshape(sb)
ns = [scale * 2 ** k for k in range(T + 1, 1, -1)]


def make():
    gp = F.FastGPLattice(d, seed_for_seq=7, num_tasks=T, shape_batch=sb, shape_scale=sb + [1],
                         shape_lengthscales=sb[1:] + [d], shape_noise=sb[2:] + [1],
                         shape_factor_task_kernel=sb + [T, T], shape_noise_task_kernel=sb[1:] + [T], device=dev)
    xs = gp.get_x_next(n=torch.tensor(ns))
    g = torch.Generator(device=dev).manual_seed(11)
    gp.add_y_next([(consts[..., None, None] * xs[l] ** torch.arange(1, d + 1, device=dev)).sum(-1)
                   + torch.randn(sb + [xs[l].shape[0]], generator=g, device=dev) / (3 + l) for l in range(T)])
    return gp


for rep in range(3):
    gp = make()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng = MtGeneralEngine(gp, 0.1, its + 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.run(0, its + 1, final_no_update=True)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    gp2 = make()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    gp2.fit(iterations=its, verbose=0, stop_crit_wait_iterations=its + 1, store_loss_hist=True)
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    print("rep %d: engine build %.3f ms, run enqueue %.3f ms, run total %.3f ms, fit %.3f ms"
          % (rep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t1), 1e3 * (t5 - t4)), flush=True)
