"""Golden vectors for the PARAMETER-BATCHED multitask GP of the reference's docs/examples/batch_multitask/fgp_lattice.ipynb
(cell 4: d = 6, shape_batch = [2, 3, 4], 5 tasks, the data function f(l, x); cell 6: shape_scale = shape_batch + [1],
shape_lengthscales = shape_batch[1:] + [d], shape_noise = shape_batch[2:] + [1], shape_factor_task_kernel =
shape_batch + [5, 5], shape_noise_task_kernel = shape_batch[1:] + [5]; cell 7: n = 2^[6, 5, 4, 3, 2] per task), from
the REAL reference (VERDICT r04 "Next round" item 6).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_batch_mt.py

The notebook's point sets come from qmcpy's default generating vector (absent offline): here the package's
committed vector and explicit shifts per task; the notebook's lattice GP otherwise as written, plus a digital-net
variant of the same shapes (d = 3, alpha = 2).  Writes tests/golden/batch_mt/*.npz: inputs (generating vector /
matrices, shifts, every task's observations [2, 3, 4, n_l], the initial raw parameters) and the reference's
outputs: the MLL and its gradient at the initial parameters, fit(iterations=4) (early stopping off) loss history and
every fitted raw parameter, post_mean / post_var at 12 test points and post_cov between 4 and 5 of them after the fit.
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
from make_golden import LATTICE_Z, _np, sobol_generating_matrices  # noqa: E402

OUT = os.path.join(HERE, "batch_mt")
ITS = 4
SHAPE_BATCH = [2, 3, 4]
T = 5
CASES = [("lattice", 6, 2), ("net", 3, 2)]
PNAMES = ("raw_scale", "raw_lengthscales", "raw_noise", "raw_factor_task_kernel", "raw_noise_task_kernel")


def data_fn(d, rng):
    """The notebook's f(l, x) (cell 4)."""
    def f(l, x):
        consts = torch.arange(int(np.prod(SHAPE_BATCH))).reshape(SHAPE_BATCH).to(torch.float64)
        return (consts[..., None, None] * x ** torch.arange(1, d + 1)).sum(-1) + \
            torch.randn(SHAPE_BATCH + [x.size(0)], generator=rng) / (3 + l)
    return f


def gen(fg, qmcpy, family, d, alpha, seed=7):
    out = {"family": np.array(family), "d": np.array(d), "alpha": np.array(alpha), "T": np.array(T),
           "shape_batch": np.array(SHAPE_BATCH)}
    kw = dict(alpha=alpha, num_tasks=T, shape_batch=SHAPE_BATCH, shape_scale=SHAPE_BATCH + [1],
              shape_lengthscales=SHAPE_BATCH[1:] + [d], shape_noise=SHAPE_BATCH[2:] + [1],
              shape_factor_task_kernel=SHAPE_BATCH + [T, T], shape_noise_task_kernel=SHAPE_BATCH[1:] + [T])
    if family == "lattice":
        shifts = np.stack([np.random.default_rng(seed + l).uniform(size=d) for l in range(T)])
        seqs = [qmcpy.Lattice(d, randomize="SHIFT", generating_vector=LATTICE_Z[:d], shift=shifts[l]) for l in range(T)]
        out["z"] = np.array(LATTICE_Z[:d], dtype=np.int64)
        out["shifts"] = shifts
        gp = fg.FastGPLattice(seqs, **kw)
    else:
        t = 32
        C = sobol_generating_matrices(d, t=t)
        shifts = np.stack([np.random.default_rng(seed + l).integers(0, 2 ** t, size=d, dtype=np.uint64) for l in range(T)])
        seqs = [qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=C, t=t, shift=shifts[l]) for l in range(T)]
        out["C"] = C.astype(np.int64)
        out["t"] = np.array(t)
        out["shifts"] = shifts.astype(np.int64)
        gp = fg.FastGPDigitalNetB2(seqs, **kw)
    for nm in PNAMES:
        out["init_" + nm] = _np(getattr(gp, nm)).copy()     # the fit steps the parameters in place
    ns = [int(v) for v in 2 ** torch.arange(T + 1, 1, -1)]
    out["ns"] = np.array(ns, dtype=np.int64)
    xs = gp.get_x_next(n=torch.tensor(ns))
    f = data_fn(d, torch.Generator().manual_seed(seed))
    ys = [f(l, xs[l]) for l in range(T)]
    gp.add_y_next(ys)
    for l in range(T):
        out["x_%d" % l] = _np(xs[l])
        out["y_%d" % l] = _np(ys[l])
    # MLL and its gradient at the initial parameters (abstract_gp.py:235,253-260,294)
    os.environ["FASTGP_FORCE_RECOMPILE"] = "True"
    cache = gp.get_inv_log_det_cache()
    norm_term, logdet = cache.get_norm_term_logdet_term()
    d_out = int(np.prod(SHAPE_BATCH))
    loss = 0.5 * (norm_term.sum() + d_out / torch.tensor(logdet.shape).prod() * logdet.sum() +
                  d_out * gp.n.sum() * np.log(2 * np.pi))
    names = [nm for nm in PNAMES if getattr(gp, nm).requires_grad]
    grads = torch.autograd.grad(loss, [getattr(gp, nm) for nm in names])
    del os.environ["FASTGP_FORCE_RECOMPILE"]
    out["loss"] = _np(loss)
    out["grad_names"] = np.array(names)
    for nm, g in zip(names, grads):
        out["grad_" + nm] = _np(g)
    data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=ITS + 5)
    out["fit_loss_hist"] = _np(data["loss_hist"])
    for nm in PNAMES:
        out["fit_" + nm] = _np(getattr(gp, nm)).copy()
    xt = torch.rand((12, d), generator=torch.Generator().manual_seed(17))
    out["x_test"] = _np(xt)
    out["fit_pmean"] = _np(gp.post_mean(xt))
    out["fit_pvar"] = _np(gp.post_var(xt))
    out["fit_pcov"] = _np(gp.post_cov(xt[:4], xt[4:9]))
    return out


def main():
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    os.makedirs(OUT, exist_ok=True)
    for family, d, alpha in CASES:
        name = "%s_d%d_a%d_T%d_b%s" % (family, d, alpha, T, "x".join(str(v) for v in SHAPE_BATCH))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **gen(fg, qmcpy, family, d, alpha))
        print("wrote", name)


if __name__ == "__main__":
    main()
