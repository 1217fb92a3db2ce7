"""A/B of the half-length real inverse (fgp_ifftbr_real_rf, the C5 coefficient solve) at 512 x 2^18: the
whole batch per launch pair vs groups of FGP_C2R_GROUP rows (the intermediate of a group can stay in the
Infinity Cache between the column and the row pass).  Prints one JSON line: ms per call (shared / per-row factor).
The FGP_C2R_GROUP hook of ifftbr_real_any was removed after the A/B (profiles/r05k_c2r_group_ab.jsonl: 1.26-1.33 ms
at every group size -- the two passes are not bound by where the intermediate lives)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from fastgaussianprocesses_amd import ops  # noqa: E402

dev = "cuda:0"
n, B = 1 << 18, 512
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn((B, n // 2 + 1), dtype=torch.complex128, device=dev, generator=g)
res = {"group": int(os.environ.get("FGP_C2R_GROUP", "0"))}
for name, f in (("shared", torch.rand((1, n), dtype=torch.float64, device=dev, generator=g) + 0.5),
                ("per_row", torch.rand((B, n), dtype=torch.float64, device=dev, generator=g) + 0.5)):
    out = ops.ifftbr_real_rf(x, f, n=n)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(6):
        ev[0].record()
        out = ops.ifftbr_real_rf(x, f, n=n)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    res[name + "_ms"] = sorted(ts)[len(ts) // 2]
    res[name + "_checksum"] = float(out[:, :1024].sum())
print(json.dumps(res), flush=True)
