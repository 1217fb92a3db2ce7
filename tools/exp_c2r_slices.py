"""A/B of the half-length real inverse (fgp_ifftbr_real_rf, the C5 coefficient solve) at 512 x 2^18 after the
column pass's loads were put in flight together (r05u): the whole batch in one launch pair vs slices of S rows
(one launch pair per slice; a slice's 2 MB-per-row intermediate can stay in the 256 MB Infinity Cache between the
column and the row pass).  Prints one JSON line per S: ms per call (median of 6, events)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from fastgaussianprocesses_amd import ops  # noqa: E402

dev = "cuda:0"
n, B = 1 << 18, 512
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn((B, n // 2 + 1), dtype=torch.complex128, device=dev, generator=g)
f = torch.rand((1, n), dtype=torch.float64, device=dev, generator=g) + 0.5
ref = ops.ifftbr_real_rf(x, f, n=n)
for S in (512, 256, 128, 64, 32, 16):
    def call():
        return [ops.ifftbr_real_rf(x[i:i + S], f, n=n) for i in range(0, B, S)]
    outs = call()
    same = all(torch.equal(o, ref[i * S:(i + 1) * S]) for i, o in enumerate(outs))
    del outs
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(6):
        ev[0].record()
        outs = call()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
        del outs
    print(json.dumps({"slice_rows": S, "ms": sorted(ts)[3], "equal_to_whole": same}), flush=True)
