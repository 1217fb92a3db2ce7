"""Host-side cost of one small fit (the probnum25 paper's protocol: n = 2^10, reference fit defaults): wall time
of gp.fit per configuration and a cProfile of the Ackley d = 1 lattice fit (the fixed costs around the
single-launch iteration loop: ytilde, spectra, engine set-up, histories).

    python tools/prof_fit_small.py [--reps 3]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    name, d, f, _ = bench.paper_functions()[0]

    def one(iterations=5000):
        gp = F.FastGPLattice(F.Lattice(d, seed=7), alpha=2, device=dev)
        xs = gp.get_x_next(1024)
        gp.add_y_next(f(xs))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        data = gp.fit(iterations=iterations, verbose=0, store_loss_hist=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, int(data["iterations"])

    one(3)
    for r in range(args.reps):
        el, its = one()
        print('{"bench": "%s", "d": %d, "iterations": %d, "fit_s": %.6f, "s_per_step": %.3e}' % (name, d, its, el, el / its),
              flush=True)
    pr = cProfile.Profile()
    gp = F.FastGPLattice(F.Lattice(d, seed=7), alpha=2, device=dev)
    xs = gp.get_x_next(1024)
    gp.add_y_next(f(xs))
    torch.cuda.synchronize()
    pr.enable()
    gp.fit(iterations=5000, verbose=0, store_loss_hist=True)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr).stats          # {(file, line, fn): (cc, nc, tottime, cumtime, callers)}
    rows = sorted(st.items(), key=lambda kv: -kv[1][3])[:60]
    print("%9s %9s %6s  %s" % ("cum_us", "self_us", "calls", "function"))
    for (fn, ln, name), (cc, nc, tt, ct, _) in rows:
        print("%9.1f %9.1f %6d  %s:%d(%s)" % (ct * 1e6, tt * 1e6, nc, os.path.basename(fn), ln, name))


if __name__ == "__main__":
    main()
