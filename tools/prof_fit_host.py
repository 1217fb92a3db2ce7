"""cProfile of one eager C2 / C3 fit (bench.SingleGP, 50 iterations): where the host time of ytilde+fit goes."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fastgaussianprocesses_amd as F  # noqa: E402

fam = sys.argv[1] if len(sys.argv) > 1 else "lattice"
sg = bench.SingleGP(F, fam, 16, 3, "cuda:0")
for _ in range(3):
    sg.reset()
    sg.gp.fit(iterations=50, stop_crit_wait_iterations=51, verbose=0)
torch.cuda.synchronize()
sg.reset()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
sg.gp.fit(iterations=50, stop_crit_wait_iterations=51, verbose=0)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
rows = sorted(st.stats.items(), key=lambda kv: -kv[1][3])
print("cumulative us  tottime us  calls  function")
for (fn, line, name), (cc, nc, tt, ct, _) in rows[:60]:
    print("%12.1f %11.1f %6d  %s:%d(%s)" % (ct * 1e6, tt * 1e6, nc, os.path.basename(fn), line, name))
