"""Where the time of the single-launch fit (fgp_fit_persist) goes: workgroup 0's device-clock stamps per
iteration (start, partials stored, barrier passed, partials reduced, Rprop applied) for C2 / C3 (n = 2^16,
d = 3) and the paper's n = 2^10 single-task fits; one JSON line per configuration with the per-phase medians
(us) and the wall time of the launch.

    python tools/exp_persist_stamps.py [--iters 50]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    khz = bench.wall_clock_khz(F, dev)
    cfgs = [("C2 lattice", "lattice", 16, 3, 2), ("C3 net", "net", 16, 3, 2), ("paper lattice d1", "lattice", 10, 1, 2),
            ("paper lattice d2", "lattice", 10, 2, 2), ("paper lattice d6", "lattice", 10, 6, 2),
            ("paper net d2", "net", 10, 2, 4)]
    it = args.iters
    for name, fam, m, d, alpha in cfgs:
        g = torch.Generator().manual_seed(3)
        if fam == "lattice":
            gp = F.FastGPLattice(F.Lattice(d, seed=7), alpha=alpha, device=dev)
        else:
            gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=7, randomize="DS"), alpha=alpha, device=dev)
        x = gp.get_x_next(2 ** m)
        gp.add_y_next(torch.sin(6 * x).sum(1) + 0.1 * torch.rand(x.shape[0], generator=g).to(dev))
        eng = gp._fused_engine(it, 0.1)
        if not eng.persist_ok():
            print(json.dumps({"config": name, "persist": False}), flush=True)
            continue
        st = torch.zeros((it + 1) * 5, dtype=torch.int64, device=dev)
        eng.run_persist(it, math.log(1.05), it + 1)      # warm
        torch.cuda.synchronize()
        eng._nll.stamps = st.data_ptr()
        t0 = time.perf_counter()
        eng.run_persist(it, math.log(1.05), it + 1)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        eng._nll.stamps = None
        s = st.reshape(it + 1, 5).double().cpu() * (1e3 / khz)
        ph = {"compute": s[:, 1] - s[:, 0], "barrier": s[:, 2] - s[:, 1], "reduce": s[:, 3] - s[:, 2],
              "step": s[:, 4] - s[:, 3]}
        out = {"config": name, "n": 2 ** m, "d": d, "iterations": it, "wall_us": 1e6 * wall,
               "device_us_per_iter": float((s[-1, 4] - s[0, 0]) / (it + 1)),
               "prologue_us_to_first": None}
        for k, v in ph.items():
            out[k + "_p50_us"] = float(v.median())
        out["next_p50_us"] = float((s[1:, 0] - s[:-1, 4]).median())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
