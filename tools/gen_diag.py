"""Diagnostic: generated lattice points / parts vs the host generator + fgp_lattice_parts, and the
fused MLL with regenerated vs array parts at random hyper-parameters."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_default_dtype(torch.float64)
import fastgaussianprocesses_amd as F  # noqa: E402
from oracle.fgp_oracle import f_ackley  # noqa: E402

for m, d, alpha in [(14, 5, 2), (16, 4, 3), (17, 4, 3), (17, 4, 2), (20, 5, 2)]:
    n = 2 ** m
    seq = F.Lattice(d, seed=11)
    xh = torch.from_numpy(seq(0, n)).cuda()
    xg = F.ops.lattice_points(seq.z[:d], seq.shift, 0, n, device="cuda")
    pa = F.ops.lattice_parts(xh, xh[0], [alpha] * d)
    pg = F.ops.lattice_parts_gen(seq.z[:d], xh[0], [alpha] * d, n)
    bad = (pa != pg).nonzero()
    print(m, d, alpha, "points equal", bool(torch.equal(xh, xg)), "n points differ", int((xh != xg).sum()),
          "parts equal", bool(torch.equal(pa, pg)), "n parts differ", bad.shape[0])
    if bad.shape[0]:
        j, i = bad[0].tolist()
        print("   first diff j=%d i=%d  x=%r x0=%r array=%r gen=%r" % (j, i, float(xh[i, j]), float(xh[0, j]),
                                                                    float(pa[j, i]), float(pg[j, i])))
    res = {}
    for mode in ("1", "0"):
        os.environ["FGP_PARTS_GEN"] = mode
        gp = F.FastGPLattice(F.Lattice(d, seed=11), alpha=alpha, device="cuda")
        gp.add_y_next(f_ackley(gp.get_x_next(n)))
        with torch.no_grad():
            g = torch.Generator().manual_seed(m * 10 + d)
            gp.raw_lengthscales.copy_(0.5 * torch.randn(gp.raw_lengthscales.shape, generator=g))
            gp.raw_scale.copy_(0.3 * torch.randn(gp.raw_scale.shape, generator=g))
            lam = gp.get_lam().clone()
        eng = F.batch.batched_engine([gp], 4)
        res[mode] = eng.evaluate() + (lam,)
    a, b = res["1"], res["0"]
    print("   loss diff", a[0] - b[0], "grad diff", (a[3] - b[3]).abs().max().item(), "lam equal",
          bool(torch.equal(a[4], b[4])))
