"""CPU-baseline fidelity: time the oracle (oracle/fgp_oracle.py, the torch-CPU
restatement that bench.py's cpu_baseline runs on the GPU box) against the REAL reference (fastgps @
/root/reference via oracle/refshim) on the same cores, for one BASELINE C4 GP (FastGPLattice
n = 2^20, d = 5, alpha = 2, shift seed 1000, y = f_ackley).  Build container only (the reference does
not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_fidelity.py [--log2n 20] [--iters 3] > profiles/r02_cpu_fidelity.json

Per phase (seconds): one-time setup (ytilde, first-column kernel parts), one fit iteration (loss +
backward + Rprop step, averaged over --iters + 1 loss evaluations),
post_mean per test point (8 points), post_var per test point (1 point); ratio = oracle / reference.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def f_ackley(x, a=20, b=0.2, c=2 * np.pi, scaling=32.768):
    x = 2 * scaling * x - scaling
    t1 = a * torch.exp(-b * torch.sqrt(torch.mean(x ** 2, 1)))
    t2 = torch.exp(torch.mean(torch.cos(c * x), 1))
    return -t1 - t2 + a + np.exp(1)


def time_fit(fit_fn, iters):
    t0 = time.perf_counter()
    fit_fn(iters)
    return (time.perf_counter() - t0) / (iters + 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    p.add_argument("--iters", type=int, default=5)
    a = p.parse_args()
    torch.set_default_dtype(torch.float64)
    n, d = 2 ** a.log2n, a.d
    from oracle import fgp_oracle as O
    from oracle.refshim.load_reference import import_reference
    from fastgaussianprocesses_amd.seqs import DEFAULT_LATTICE_Z
    fg = import_reference()
    import qmcpy
    z = DEFAULT_LATTICE_Z[:d]
    shift = np.random.default_rng(1000).uniform(size=d)
    g = torch.Generator().manual_seed(17)
    xm = torch.rand((8, d), generator=g)
    xv = torch.rand((1, d), generator=g)
    res = {"config": "FastGPLattice n=2^%d d=%d alpha=2 (BASELINE C4, one GP)" % (a.log2n, d),
           "threads": torch.get_num_threads(), "fit_iters_timed": a.iters}
    # the reference
    ref = fg.FastGPLattice(qmcpy.Lattice(d, randomize="SHIFT", generating_vector=z, shift=shift))
    x = ref.get_x_next(n)
    y = f_ackley(x)
    ref.add_y_next(y)
    t0 = time.perf_counter()
    ref.get_ytilde(0)
    ref.get_k1parts(0, 0)            # one-time parts (cached across fit iterations, as the oracle's)
    t_setup_ref = time.perf_counter() - t0
    t_fit_ref = time_fit(lambda k: ref.fit(iterations=k, verbose=0, stop_crit_wait_iterations=k + 1), a.iters)
    t0 = time.perf_counter()
    ref.coeffs
    t_coeffs_ref = time.perf_counter() - t0
    t0 = time.perf_counter()
    pm_ref = ref.post_mean(xm)
    t_pm_ref = (time.perf_counter() - t0) / len(xm)
    t0 = time.perf_counter()
    ref.post_var(xv)
    t_pv_ref = time.perf_counter() - t0
    # the oracle on the same points and data
    o = O.OracleFastGP("lattice", x, None, y, alpha=2)
    t0 = time.perf_counter()
    o.ytilde()
    o.k1parts()
    t_setup_o = time.perf_counter() - t0
    t_fit_o = time_fit(lambda k: o.fit(iterations=k, stop_crit_wait_iterations=k + 1), a.iters)
    t0 = time.perf_counter()
    o.coeffs()
    t_coeffs_o = time.perf_counter() - t0
    t0 = time.perf_counter()
    pm_o = o.post_mean(xm, chunk=4)
    t_pm_o = (time.perf_counter() - t0) / len(xm)
    t0 = time.perf_counter()
    o.post_var(xv)
    t_pv_o = time.perf_counter() - t0
    phases = {}
    for name, tr, to in (("setup (ytilde, parts)", t_setup_ref, t_setup_o), ("fit_iteration", t_fit_ref, t_fit_o),
                         ("coeffs", t_coeffs_ref, t_coeffs_o), ("post_mean_per_point", t_pm_ref, t_pm_o),
                         ("post_var_per_point", t_pv_ref, t_pv_o)):
        phases[name] = {"reference_s": tr, "oracle_s": to, "oracle_over_reference": to / tr}
    res["phases"] = phases
    # the bench step's per-GP workload (50 fit iterations + post_mean N=256 + post_var N=8)
    step = lambda ph, k: (ph["setup (ytilde, parts)"][k] + 51 * ph["fit_iteration"][k] + ph["coeffs"][k] +
                          256 * ph["post_mean_per_point"][k] + 8 * ph["post_var_per_point"][k])
    res["bench_step_per_gp"] = {"reference_s": step(phases, "reference_s"), "oracle_s": step(phases, "oracle_s")}
    res["port_vs_reference"] = res["bench_step_per_gp"]["oracle_s"] / res["bench_step_per_gp"]["reference_s"]
    res["post_mean_max_rel_diff"] = float((pm_ref - pm_o).abs().max() / pm_ref.abs().max())
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
