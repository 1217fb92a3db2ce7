"""Spectral iteration for many problems on one set of spectra (C5 per-output hyper-parameters: 512
eigen-problems, n = 2^18, d = 3): the per-wave kernel k_spec_iter (FGP_SPEC_TILE=0) against the tile kernel
over problem slices at several k-block counts (FGP_SPEC_SLICE_NB) (and ring depths: the FGP_SPEC_SLICE_RING
switch of the measured build was removed after profiles/r03sl_exp_slices.jsonl showed no gain).  Per variant: the iteration kernel alone
(FusedMLL.stage) and the staged fit loop per iteration (FusedMLL.run: kernel + k_spec_reduce_step).  HIP
events on torch's current stream; one JSON line per variant.

    python tools/exp_slices.py [--log2n 18] [--d 3] [--outputs 512] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def ev_time(fn, reps=1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2e6))
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=18)
    ap.add_argument("--d", type=int, default=3)
    ap.add_argument("--outputs", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nbs", default="128,64,32,16")
    ap.add_argument("--rings", default="2")
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    os.environ["FGP_FIT_PATH"] = "spectral"
    sg = bench.MultiOutputGP(F, args.log2n, args.d, args.outputs, dev, per_output=True)
    sg.reset()
    variants = [("per-wave k_spec_iter", {"FGP_SPEC_TILE": "0"})]
    variants += [("tile slices default geometry", {"FGP_SPEC_TILE": "1"})]
    variants += [("tile slices nb=%s ring=%s" % (nb, r), {"FGP_SPEC_TILE": "1", "FGP_SPEC_SLICE_NB": nb,
                                                          "FGP_SPEC_SLICE_RING": r})
                 for r in args.rings.split(",") for nb in args.nbs.split(",")]
    ref = None
    for name, env in variants:
        os.environ.pop("FGP_SPEC_SLICE_NB", None)
        os.environ.pop("FGP_SPEC_SLICE_RING", None)
        os.environ.update(env)
        eng = sg.gp._fused_engine(args.iters, 0.1)
        eng.run(0, 2)
        torch.cuda.synchronize()
        t_stage = ev_time(lambda: eng.stage(0), 20)
        loss = eng.evaluate()[0]
        it = args.iters
        t_run = ev_time(lambda: eng.run(0, it)) / it
        ref = loss if ref is None else ref
        print(json.dumps({"variant": name, "stage_us": 1e3 * t_stage, "fit_run_us_per_iter": 1e3 * t_run,
                          "loss_rel_vs_first": abs(loss - ref) / abs(ref)}), flush=True)
    os.environ.pop("FGP_SPEC_SLICE_NB", None)
    os.environ.pop("FGP_SPEC_TILE", None)


if __name__ == "__main__":
    main()
