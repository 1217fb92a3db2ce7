"""Diagnostic: loss terms and gradient of the fused MLL with regenerated vs array lattice parts."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.set_default_dtype(torch.float64)
import fastgaussianprocesses_amd as F  # noqa: E402
from oracle.fgp_oracle import f_ackley  # noqa: E402

for m, d, alpha in [(14, 5, 2), (17, 4, 3), (17, 4, 2), (13, 3, 4), (16, 2, 1)]:
    res = {}
    for mode in ("1", "0"):
        os.environ["FGP_PARTS_GEN"] = mode
        gp = F.FastGPLattice(F.Lattice(d, seed=11), alpha=alpha, device="cuda")
        gp.add_y_next(f_ackley(gp.get_x_next(2 ** m)))
        with torch.no_grad():
            g = torch.Generator().manual_seed(m * 10 + d)
            gp.raw_lengthscales.copy_(0.5 * torch.randn(gp.raw_lengthscales.shape, generator=g))
            gp.raw_scale.copy_(0.3 * torch.randn(gp.raw_scale.shape, generator=g))
            lam = gp.get_lam().clone()
        eng = F.batch.batched_engine([gp], 4)
        res[mode] = eng.evaluate() + (lam,)
    a, b = res["1"], res["0"]
    print(m, d, alpha, "loss diff", a[0] - b[0], "norm diff", a[1] - b[1], "logdet diff", a[2] - b[2],
          "grad diff", (a[3] - b[3]).tolist(), "lam equal", bool(torch.equal(a[4], b[4])))
