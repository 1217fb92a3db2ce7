"""(Historical: the FGP_SPEC_EXP_NOCOMPUTE switch these runs used was removed from the product kernel
after the round-3 measurements; its 'stream' rows need a build of commit e26f9e6.)
Tile-kernel ring-depth / LDS variants (experiment builds, tools/build_exp.sh into _lib/exp/): for each
library, the C4-shaped iteration kernel (8 GPs sharing one set of spectra, n = 2^20, d = 5) streaming only
(FGP_SPEC_EXP_NOCOMPUTE=1) and complete, HIP events.  One JSON line per variant.

    python tools/exp_spec_ring.py lib1.so lib2.so ...   (in-tree library when none given)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, %r)
torch.set_default_dtype(torch.float64)
import bench
import fastgaussianprocesses_amd as F
from fastgaussianprocesses_amd.fit_engine import FusedMLL, mll_constant
dev = torch.device("cuda", 0)
n, d = 2 ** 20, 5
sh = bench.Shifts(F, d, n, bench.shard_seeds(0, 1, 8), dev)
sh.reset()
b = sh.batch
bas = b.basis()
raw = b.raw()
def t(fn, reps=20):
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize()
    a.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(e) / reps
out = {"lib": os.environ.get("FGP_LIB_PATH", "in-tree")}
for mode in ("stream", "full"):
    os.environ["FGP_SPEC_EXP_NOCOMPUTE"] = "1" if mode == "stream" else "0"
    e8 = FusedMLL(0, None, b.ysq(), raw[:, 0], raw[:, 1:1 + d], raw[:, -1], 1.0, mll_constant(1, n),
                  max_iters=64, per_problem=True, basis=bas)
    out[mode + "_us"] = t(lambda: e8.stage(0))
    if mode == "full":
        out["fit_run_us_per_iter"] = t(lambda: e8.run(0, 50), 2) / 50
print(json.dumps(out), flush=True)
''' % ROOT


def main():
    libs = sys.argv[1:] or [None]
    for lib in libs:
        env = dict(os.environ)
        if lib:
            env["FGP_LIB_PATH"] = lib
        env["FGP_FIT_PATH"] = "spectral"
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           timeout=240)
        sys.stdout.write(r.stdout.decode())
        if r.returncode != 0:
            sys.stdout.write(json.dumps({"lib": lib, "error": r.stderr.decode()[-800:]}) + "\n")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
