"""Why does k_spec_tile run ~37 us per launch inside the timed C4 step but ~40 us timed on its own?  The C4 batch's
fit (fgp_fit_run, 50 iterations) captured once into a hipGraph and replayed (A) back to back, (B) each replay behind
an in-place rewrite of the 134 MB of spectra it streams (the lines freshly written, as after the step's spectra
build), (C) behind a 537 MB write to an unrelated buffer (as post_var's intermediate).  Two k_clock_stamp launches
separate the three loops in a rocprofv3 --kernel-trace; prints the per-loop averages from the trace is left to
the caller (tools/timed_region_stats.py-style split on the markers).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o t -- python3 tools/exp_fit_after_basis.py
"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fastgaussianprocesses_amd as F  # noqa: E402

dev = torch.device("cuda", 0)
n, d, iters = 1 << 20, 5, 50
sh = bench.Shifts(F, d, n, list(range(1000, 1008)), dev)
sh.reset()
eng = F.batch.batched_engine(sh.gps, iters)
assert eng.basis is not None
basis = eng.basis
tmp = torch.empty_like(basis)
junk = torch.empty((537 << 20) // 8, dtype=torch.float64, device=dev)
eng.run(0, iters)
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        eng.run(0, iters)
torch.cuda.current_stream().wait_stream(s)
marks = torch.zeros(4, dtype=torch.int64, device=dev)


def mark(i):
    F._native.call("fgp_clock_stamp", marks[i:i + 1].data_ptr(), torch.cuda.current_stream().cuda_stream)


g.replay()
torch.cuda.synchronize()
mark(0)
for _ in range(3):                     # (A) back to back
    g.replay()
mark(1)
for _ in range(3):                     # (B) behind a rewrite of the spectra
    tmp.copy_(basis)
    basis.copy_(tmp)
    g.replay()
mark(2)
for _ in range(3):                     # (C) behind a 537 MB write elsewhere
    junk.fill_(1.0)
    g.replay()
mark(3)
torch.cuda.synchronize()
print("done", flush=True)
