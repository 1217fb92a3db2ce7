"""Shared helpers for the GPU parity tests: build product GPs from the golden fixtures."""
import numpy as np
import torch

import fastgaussianprocesses_amd as F

DEV = "cuda"


def product_gp(g, **kw):
    fam = str(g["family"])
    d = int(g["d"])
    B = int(g["B"])
    extra = dict(kw)
    if B > 0:
        extra["shape_batch"] = [B]
    if bool(g["per_output"]):
        extra["shape_scale"] = [B, 1]
        extra["shape_lengthscales"] = [B, d]
    if fam == "lattice":
        seq = F.Lattice(d, randomize="SHIFT", generating_vector=g["z"], shift=g["shift"])
        gp = F.FastGPLattice(seq, alpha=int(g["alpha"]), device=DEV, **extra)
    else:
        seq = F.DigitalNetB2(d, randomize="DS", generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                             shift=g["shift"].astype(np.uint64))
        gp = F.FastGPDigitalNetB2(seq, alpha=int(g["alpha"]), device=DEV, **extra)
    n = 2 ** int(g["m"])
    x = gp.get_x_next(n)
    assert np.array_equal(x.cpu().numpy(), g["x"]), "point generation differs from the reference fixture"
    gp.add_y_next(torch.from_numpy(g["y"]).to(DEV))
    return gp


def rel_err(a, b):
    a = torch.as_tensor(a).detach().cpu().reshape(-1)
    b = (b.detach().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b))).reshape(-1)
    if b.numel() == 0:
        return 0.0
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-300)


def abs_err(a, b):
    a = torch.as_tensor(a).detach().cpu().reshape(-1)
    b = (b.detach().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b))).reshape(-1)
    return float((a - b).abs().max()) if b.numel() else 0.0
