"""Golden vectors for the EXACT benched C4 work (BASELINE config C4: FastGPLattice n = 2^20, d = 5, alpha = 2,
the default nugget 1e-8; bench.py's step: fit 50 Rprop iterations with early stopping off, then post_mean and
post_var) from the REAL reference, for two of bench.py's shifts, and the reference's own FFT-backend spread
over those 50 iterations (VERDICT r04 "Next round" item 1).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c4.py

Writes tests/golden/c4_m20_d5_it50.npz: per shift seed (1000, 1001 -- bench.shard_seeds(0, 1, 8)[:2]) the
inputs (generating vector z, the shift default_rng(seed).uniform(size=5), the test points) and the reference's
outputs (fit(iterations=50, stop_crit_wait_iterations=51) loss history, fitted raw parameters, post_mean at 16
test points, post_var at the first 2, K(x, x) at those), and profiles/r05_c4_backend_spread.json: the same
runs with the reference's qmcpy fftbr_torch / ifftbr_torch replaced by numpy's pocketfft (make_golden_c5's
differentiable wrappers) -- the spread a correct implementation of the reference shows over this trajectory.
tests/test_gpu_bench_path.py::test_bench_step_50_iterations_matches_reference allows 5x it.
Only arrays go into the fixture (inputs and reference outputs); y = f_ackley(x) is recomputed by the test.
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from oracle.refshim.load_reference import import_reference  # noqa: E402
from make_golden import LATTICE_Z, f_ackley  # noqa: E402
from make_golden_c5 import _NpFFTBR, _NpIFFTBR, rel  # noqa: E402

M, D, ITS, NM, NV = 20, 5, 50, 16, 2
SEEDS = (1000, 1001)


def run(fg, qmcpy, seed):
    """bench.Shifts + bench.step_batched for one shift, through the reference (abstract_gp.py:152-416)."""
    n = 2 ** M
    shift = np.random.default_rng(seed).uniform(size=D)
    seq = qmcpy.Lattice(D, randomize="SHIFT", generating_vector=LATTICE_Z[:D], shift=shift)
    gp = fg.FastGPLattice(seq, alpha=2)
    x = gp.get_x_next(n)
    gp.add_y_next(f_ackley(x))
    t0 = time.perf_counter()
    data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=ITS + 1)
    t_fit = time.perf_counter() - t0
    xt = torch.rand((NM, D), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt)
    pv = gp.post_var(xt[:NV])
    out = dict(shift=shift, x_test=xt.numpy(), loss_hist=data["loss_hist"].detach().numpy(),
               raw_scale=gp.raw_scale.detach().numpy().reshape(-1),
               raw_lengthscales=gp.raw_lengthscales.detach().numpy().reshape(-1),
               pmean=pm.detach().numpy(), pvar=pv.detach().numpy(),
               kxx=gp.kernel(xt[:NV], xt[:NV]).detach().numpy().reshape(-1))
    print("seed %d: fit %.1f s, final loss %.6f" % (seed, t_fit, float(out["loss_hist"][-1])), flush=True)
    return out


def main():
    torch.set_default_dtype(torch.float64)
    torch.set_num_threads(os.cpu_count() or 1)
    fg = import_reference()
    import qmcpy
    keep = (qmcpy.fftbr_torch, qmcpy.ifftbr_torch)
    ref = [run(fg, qmcpy, s) for s in SEEDS]
    qmcpy.fftbr_torch, qmcpy.ifftbr_torch = _NpFFTBR.apply, _NpIFFTBR.apply
    alt = [run(fg, qmcpy, s) for s in SEEDS]
    qmcpy.fftbr_torch, qmcpy.ifftbr_torch = keep
    st = lambda rs, k: np.stack([r[k] for r in rs])
    keys = ("shift", "loss_hist", "raw_scale", "raw_lengthscales", "pmean", "pvar", "kxx")
    np.savez_compressed(os.path.join(HERE, "c4_m20_d5_it50.npz"), m=np.array(M), d=np.array(D), its=np.array(ITS),
                        z=np.array(LATTICE_Z[:D], dtype=np.int64), seeds=np.array(SEEDS, dtype=np.int64),
                        x_test=ref[0]["x_test"], **{k: st(ref, k) for k in keys})
    lh_r, lh_a = st(ref, "loss_hist"), st(alt, "loss_hist")
    spread = {"config": "C4 one GPU's share, per shift: lattice n=2^%d d=%d alpha=2, nugget 1e-8, fit(iterations=%d, "
                        "stop_crit_wait_iterations=%d), post_mean N=%d, post_var N=%d; shift seeds %s"
                        % (M, D, ITS, ITS + 1, NM, NV, list(SEEDS)),
              "what": "the REAL reference (tests/golden/make_golden_c4.py) with qmcpy.fftbr_torch/ifftbr_torch "
                      "(torch.fft) vs numpy pocketfft",
              "loss_hist_rel": rel(lh_a, lh_r),
              "loss_hist_rel_per_iteration_max": float(np.max(np.abs(lh_a - lh_r) / np.abs(lh_r))),
              "raw_lengthscales_abs": float(np.max(np.abs(st(alt, "raw_lengthscales") - st(ref, "raw_lengthscales")))),
              "raw_scale_abs": float(np.max(np.abs(st(alt, "raw_scale") - st(ref, "raw_scale")))),
              "pmean_rel": rel(st(alt, "pmean"), st(ref, "pmean")),
              "pvar_abs_over_kxx": float(np.max(np.abs(st(alt, "pvar") - st(ref, "pvar")) / st(ref, "kxx")))}
    with open(os.path.join(ROOT, "profiles", "r05_c4_backend_spread.json"), "w") as f:
        json.dump(spread, f, indent=1)
    print(json.dumps(spread, indent=1))


if __name__ == "__main__":
    main()
