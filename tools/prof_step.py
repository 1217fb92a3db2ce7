import cProfile, pstats, sys, os, io, time
sys.path.insert(0, os.getcwd())
import torch
torch.set_default_dtype(torch.float64)
import bench
import fastgaussianprocesses_amd as F
dev = torch.device("cuda", 0)
sh = bench.Shifts(F, 5, 2 ** 20, [1000 + s for s in range(8)], dev)
g = torch.Generator().manual_seed(3)
xm = torch.rand((256, 5), generator=g).to(dev)
xv = torch.rand((8, 5), generator=g).to(dev)
class A: fit_iters = 50
for _ in range(2): bench.step_batched(sh, A, xm, xv)
torch.cuda.synchronize()
t0 = time.perf_counter()
pr = cProfile.Profile(); pr.enable()
bench.step_batched(sh, A, xm, xv)
pr.disable()
t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
print("host enqueue %.3f ms, until GPU done %.3f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(35); print(s.getvalue()[:6000])
