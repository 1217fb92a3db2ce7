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
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
