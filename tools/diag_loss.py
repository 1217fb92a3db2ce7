"""Diagnostic: MLL trajectories through the fused fit kernels vs the generic autograd path vs the
CPU oracle, for lattice / net (alpha=1) at several sizes and dimensions."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.set_default_dtype(torch.float64)
import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O

for family, m, d in [("lattice", 13, 3), ("lattice", 17, 2), ("lattice", 17, 3), ("lattice", 18, 5), ("net", 13, 3)]:
    n = 2 ** m
    gp = F.FastGPLattice(F.Lattice(d, seed=7), device="cuda") if family == "lattice" else \
        F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=7), alpha=1, device="cuda")
    x = gp.get_x_next(n)
    y = O.f_ackley(x.cpu())
    gp.add_y_next(y.cuda())
    lg = gp._loss_generic("MLL", None, 1, 1)[0].item()
    data = gp.fit(iterations=2, store_hists=True, verbose=0, stop_crit_wait_iterations=10)
    o = O.OracleFastGP(family, x.cpu(), gp.get_xb().cpu() if family == "net" else None, y, alpha=gp._alphas[0],
                       t=getattr(gp, "t", None))
    lo = o.mll_loss()[0].item()
    print(family, m, d, "generic %.10e oracle %.10e fused-fit" % (lg, lo), data["loss_hist"].tolist(), flush=True)
