"""Golden vectors for fit(loss_metric="GCV" / "CV") of MULTITASK GPs whose task kernel is LEARNED (the reference's
default for num_tasks > 1: K_task = F F^T + diag(v), rank 1, abstract_gp.py:116-139) with equal n per task, from the
REAL reference (util.py:371-394, abstract_gp.py:242-272):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mt_learn.py

Writes tests/golden/mt_learn/<family>_d2_T3_n64.npz: the inputs (the multitask fixtures' layout: family, kind, d,
alpha, ns, B, z / C + t, shifts, x_<l>, y_<l>, x_test) and, per metric, the 6-iteration fit's loss / scale /
lengthscale / task-kernel histories, the fitted raw parameters and post_mean at x_test after the fit.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from oracle.refshim.load_reference import import_reference  # noqa: E402
from make_golden import LATTICE_Z, sobol_generating_matrices, _np  # noqa: E402
from make_golden_multitask import _fs_multitask  # noqa: E402

ITS = 6
CASES = [("lattice", 2, 2), ("net", 2, 2)]
NS = [64, 64, 64]


def build(fg, qmcpy, family, d, alpha, seed=23):
    T = len(NS)
    out = {"family": np.array(family), "kind": np.array("mt"), "d": np.array(d), "alpha": np.array(alpha),
           "ns": np.array(NS, dtype=np.int64), "B": np.array(0)}
    kw = dict(alpha=alpha, num_tasks=T)
    if family == "lattice":
        shifts = np.stack([np.random.default_rng(seed + l).uniform(size=d) for l in range(T)])
        seqs = [qmcpy.Lattice(d, randomize="SHIFT", generating_vector=LATTICE_Z[:d], shift=shifts[l]) for l in range(T)]
        out["z"] = np.array(LATTICE_Z[:d], dtype=np.int64)
        out["shifts"] = shifts
        gp = fg.FastGPLattice(seqs, **kw)
    else:
        t = 32
        C = sobol_generating_matrices(d, t=t)
        shifts = np.stack([np.random.default_rng(seed + l).integers(0, 2 ** t, size=d, dtype=np.uint64)
                           for l in range(T)])
        seqs = [qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=C, t=t, shift=shifts[l]) for l in range(T)]
        out["C"] = C.astype(np.int64)
        out["t"] = np.array(t)
        out["shifts"] = shifts.astype(np.int64)
        gp = fg.FastGPDigitalNetB2(seqs, **kw)
    xs = gp.get_x_next(n=list(NS))
    fs = _fs_multitask(d)[:T]
    ys = [fs[l](xs[l]) for l in range(T)]
    gp.add_y_next(ys)
    for l in range(T):
        out["x_%d" % l] = _np(xs[l])
        out["y_%d" % l] = _np(ys[l])
    out["x_test"] = np.random.default_rng(seed + 99).uniform(size=(7, d))
    return gp, out


def main():
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    os.makedirs(os.path.join(HERE, "mt_learn"), exist_ok=True)
    for family, d, alpha in CASES:
        out = None
        for metric in ("GCV", "CV"):
            gp, base = build(fg, qmcpy, family, d, alpha)
            out = base if out is None else out
            assert gp.raw_factor_task_kernel.requires_grad and gp.raw_noise_task_kernel.requires_grad
            data = gp.fit(loss_metric=metric, iterations=ITS, store_hists=True, verbose=0,
                          stop_crit_wait_iterations=ITS + 5)
            pre = metric.lower() + "_"
            for k in ("loss_hist", "scale_hist", "lengthscales_hist", "noise_hist", "task_kernel_hist"):
                if k in data:
                    out[pre + k] = _np(data[k])
            for k in ("raw_scale", "raw_lengthscales", "raw_noise", "raw_factor_task_kernel", "raw_noise_task_kernel"):
                out[pre + k] = _np(getattr(gp, k))
            out[pre + "pmean"] = _np(gp.post_mean(torch.from_numpy(out["x_test"])))
            print(family, metric, out[pre + "loss_hist"][:3])
        fn = os.path.join(HERE, "mt_learn", "%s_d%d_T%d_n%d.npz" % (family, d, len(NS), NS[0]))
        np.savez_compressed(fn, **out)
        print("wrote", fn)


if __name__ == "__main__":
    main()
