"""cProfile of MtGeneralEngine construction (the host side of a parameter-batched multitask fit)."""
import cProfile
import pstats
import sys

import torch

sys.path.insert(0, ".")
sys.argv = [sys.argv[0], "1"]
sys.path.insert(0, "tools")
import prof_batch_mt as P  # noqa: E402  (runs its timing loop once)
from fastgaussianprocesses_amd.multitask import MtGeneralEngine  # noqa: E402

gp = P.make()
MtGeneralEngine(gp, 0.1, 41)
gp = P.make()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
MtGeneralEngine(gp, 0.1, 41)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
rows = sorted(st.stats.items(), key=lambda kv: -kv[1][3])
print("cumulative us  tottime us  calls  function")
for (fn, line, name), (cc, nc, tt, ct, _) in rows[:45]:
    print("%12.1f %11.1f %6d  %s:%d(%s)" % (ct * 1e6, tt * 1e6, nc, fn.split("/")[-1], line, name))
