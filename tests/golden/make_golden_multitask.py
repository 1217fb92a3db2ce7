"""Golden vectors for MULTITASK and DERIVATIVE-INFORMED fast GPs, from the REAL reference.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_multitask.py [fixture names...]

Same import route as make_golden.py (oracle/refshim: in-memory PEP-646 rewrite + qmcpy stand-in); point
sets are explicit per task (one generating vector / matrix set, one shift per task) and stored in each
fixture.  The cases follow the reference's own examples: docs/examples/multitask/fgp_lattice.ipynb
(T = 3 tasks, n = [64, 8, 256], default rank-1 task kernel) and
docs/examples/derivative_informed/fgp_lattice.ipynb / fgp_dnb2.ipynb ((f, df/dx0, df/dx1), d = 2,
n = [64, 8, 256], lattice alpha = 2, net alpha = 4).

What each fixture pins (reference file:line):
  k1parts_<a><b>, lam_<a><b>   (at n = max(n_a, n_b)) _K1PartsSeq with derivative multi-indices (util.py:40-62,
                               abstract_fast_gp.py:173-180), _LamCaches (util.py:95-132) per task pair
  ytilde_<l>                   _YtildeCache per task (util.py:164-183)
  inv, logdet, norm_term       _FastInverseLogDetCache block-Schur recursion (util.py:275-337,364-370)
  loss, grad_*                 fit's MLL (abstract_gp.py:235,253-260) + autograd (:294) incl. the
                               task-kernel parameters
  coeffs                       gram_matrix_solve (util.py:338-353)
  pmean, pvar, pcov            post_mean / post_var / post_cov over all tasks (abstract_gp.py:352-474)
  pcmean, pcvar, pccov         post_cubature_* (abstract_fast_gp.py:65-154)
  pvar_new, pcvar_new          projections at n_new = n * [4, 2, 8] (abstract_fast_gp.py:41-52)
  fit_*                        fit(iterations=3, store_hists=True) trajectory (abstract_gp.py:152-306)
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
from make_golden import LATTICE_Z, sobol_generating_matrices, f_ackley, _np  # noqa: E402


def _fs_multitask(d):
    # docs/examples/multitask/fgp_lattice.ipynb cell 3: low / high fidelity Ackley and a cosine sum
    return [lambda x: f_ackley(x, c=0), lambda x: f_ackley(x), lambda x: torch.cos(2 * np.pi * x).sum(1)]


def _fs_derivative():
    # docs/examples/derivative_informed/fgp_lattice.ipynb cell 3 (d = 2)
    f = lambda x: x[:, 1] * torch.sin(x[:, 0]) + x[:, 0] * torch.cos(x[:, 1])            # noqa: E731
    f0 = lambda x: x[:, 1] * torch.cos(x[:, 0]) + torch.cos(x[:, 1])                     # noqa: E731
    f1 = lambda x: torch.sin(x[:, 0]) - x[:, 0] * torch.sin(x[:, 1])                     # noqa: E731
    return [f, f0, f1]


def gen_case(fg, qmcpy, family, kind, d, alpha, ns, B=0, seed=11, fit_its=3):
    T = len(ns)
    out = {"family": np.array(family), "kind": np.array(kind), "d": np.array(d), "alpha": np.array(alpha),
           "ns": np.array(ns, dtype=np.int64), "B": np.array(B)}
    shape_batch = [B] if B > 0 else []
    kw = dict(alpha=alpha, num_tasks=T, shape_batch=shape_batch)
    if kind == "deriv":
        assert d == 2 and T == 3
        derivs = [torch.tensor([0, 0]), torch.tensor([1, 0]), torch.tensor([0, 1])]
        kw["derivatives"] = derivs
        out["derivatives"] = np.stack([v.numpy() for v in derivs])
        fs = _fs_derivative()
    else:
        fs = _fs_multitask(d)[:T]
    seqs = []
    if family == "lattice":
        shifts = np.stack([np.random.default_rng(seed + l).uniform(size=d) for l in range(T)])
        for l in range(T):
            seqs.append(qmcpy.Lattice(d, randomize="SHIFT", generating_vector=LATTICE_Z[:d], shift=shifts[l]))
        out["z"] = np.array(LATTICE_Z[:d], dtype=np.int64)
        out["shifts"] = shifts
        fgp = fg.FastGPLattice(seqs, **kw)
    else:
        t = 32
        C = sobol_generating_matrices(d, t=t)
        shifts = np.stack([np.random.default_rng(seed + l).integers(0, 2 ** t, size=d, dtype=np.uint64)
                           for l in range(T)])
        for l in range(T):
            seqs.append(qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=C, t=t, shift=shifts[l]))
        out["C"] = C.astype(np.int64)
        out["t"] = np.array(t)
        out["shifts"] = shifts.astype(np.int64)
        fgp = fg.FastGPDigitalNetB2(seqs, **kw)
    xs = fgp.get_x_next(n=list(ns))
    ys = []
    for l in range(T):
        y = fs[l](xs[l])
        if B > 0:
            y = torch.stack([y * (1 + 0.1 * b) + 0.01 * b for b in range(B)], 0)
        ys.append(y)
    fgp.add_y_next(ys)
    for l in range(T):
        out["x_%d" % l] = _np(xs[l])
        out["xb_%d" % l] = _np(fgp.get_xb(l))
        out["y_%d" % l] = _np(ys[l])
    # per task pair caches at the initial hyper-parameters (pairs l0 <= l1, lam at n = n[l0])
    for l0 in range(T):
        for l1 in range(l0, T):
            out["k1parts_%d%d" % (l0, l1)] = _np(fgp.get_k1parts(l0, l1, n=max(ns[l0], ns[l1])))
            out["lam_%d%d" % (l0, l1)] = _np(fgp.get_lam(l0, l1, n=max(ns[l0], ns[l1])))
        out["ytilde_%d" % l0] = _np(fgp.get_ytilde(l0))
    out["gram_matrix_tasks"] = _np(fgp.gram_matrix_tasks)
    params = [p for p in (fgp.raw_scale, fgp.raw_lengthscales, fgp.raw_noise, fgp.raw_factor_task_kernel,
                          fgp.raw_noise_task_kernel) if p.requires_grad]
    names = [nm for nm, p in (("raw_scale", fgp.raw_scale), ("raw_lengthscales", fgp.raw_lengthscales),
                              ("raw_noise", fgp.raw_noise), ("raw_factor_task_kernel", fgp.raw_factor_task_kernel),
                              ("raw_noise_task_kernel", fgp.raw_noise_task_kernel)) if p.requires_grad]
    out["grad_names"] = np.array(names)
    os.environ["FASTGP_FORCE_RECOMPILE"] = "True"
    cache = fgp.get_inv_log_det_cache()
    inv, logdet0 = cache()
    out["inv"] = _np(inv)
    norm_term, logdet = cache.get_norm_term_logdet_term()
    d_out = int(torch.tensor(fgp.shape_batch).prod())
    mll_const = d_out * fgp.n.sum() * np.log(2 * np.pi)
    term1 = norm_term.sum()
    term2 = d_out / torch.tensor(logdet.shape).prod() * logdet.sum()
    loss = 0.5 * (term1 + term2 + mll_const)
    grads = torch.autograd.grad(loss, params)
    del os.environ["FASTGP_FORCE_RECOMPILE"]
    out["norm_term"] = _np(norm_term)
    out["logdet"] = _np(logdet)
    out["loss"] = _np(loss)
    for nm, g in zip(names, grads):
        out["grad_" + nm] = _np(g)
    # predictions over all tasks
    gt = torch.Generator().manual_seed(17)
    xt = torch.rand((12, d), generator=gt)
    out["x_test"] = _np(xt)
    out["coeffs"] = _np(fgp.coeffs)
    out["pmean"] = _np(fgp.post_mean(xt))
    out["pvar"] = _np(fgp.post_var(xt))
    out["pcov"] = _np(fgp.post_cov(xt[:4], xt[4:9]))
    out["pcmean"] = _np(fgp.post_cubature_mean())
    out["pcvar"] = _np(fgp.post_cubature_var())
    out["pccov"] = _np(fgp.post_cubature_cov())
    n_new = fgp.n * torch.tensor([4, 2, 8][:T])
    out["n_new"] = _np(n_new)
    out["pvar_new"] = _np(fgp.post_var(xt, n=n_new))
    out["pcvar_new"] = _np(fgp.post_cubature_var(n=n_new))
    # fit trajectory
    data = fgp.fit(iterations=fit_its, store_hists=True, verbose=0, stop_crit_wait_iterations=fit_its + 5)
    out["fit_iterations"] = np.array(data["iterations"])
    for k in ("loss_hist", "scale_hist", "lengthscales_hist", "task_kernel_hist"):
        out["fit_" + k] = _np(data[k])
    out["fit_pmean"] = _np(fgp.post_mean(xt))
    out["fit_pvar"] = _np(fgp.post_var(xt))
    return out


CASES = [
    # name, family, kind, d, alpha, ns, B
    ("mt_lattice_d1_a2_T3", "lattice", "multitask", 1, 2, [64, 8, 256], 0),
    ("mt_lattice_d2_a2_T2_b2", "lattice", "multitask", 2, 2, [32, 128], 2),
    ("mt_net_d2_a2_T3", "net", "multitask", 2, 2, [64, 8, 256], 0),
    ("deriv_lattice_d2_a2", "lattice", "deriv", 2, 2, [64, 8, 256], 0),
    ("deriv_net_d2_a4", "net", "deriv", 2, 4, [64, 8, 256], 0),
    ("deriv_lattice_d2_a3_equal", "lattice", "deriv", 2, 3, [128, 128, 128], 0),
    # equal n per task: the probnum25 paper's (f, grad f) setting (docs/examples/probnum25_paper cell 15,
    # SI lattice alpha = 2 / DSI net alpha = 4), the device-resident multitask fit's domain (8 iterations)
    ("deriv_lattice_d2_a2_equal", "lattice", "deriv", 2, 2, [256, 256, 256], 0),
    ("deriv_net_d2_a4_equal", "net", "deriv", 2, 4, [128, 128, 128], 0),
    # the paper's n = 2^10 per task (12-iteration trajectories)
    ("deriv_lattice_d2_a2_equal_n1024", "lattice", "deriv", 2, 2, [1024, 1024, 1024], 0),
    ("deriv_net_d2_a4_equal_n1024", "net", "deriv", 2, 4, [1024, 1024, 1024], 0),
]
FIT_ITS = {"deriv_lattice_d2_a2_equal": 8, "deriv_net_d2_a4_equal": 8, "deriv_lattice_d2_a2_equal_n1024": 12,
           "deriv_net_d2_a4_equal_n1024": 12}


def main():
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    only = set(sys.argv[1:])
    for name, family, kind, d, alpha, ns, B in CASES:
        if only and name not in only:
            continue
        out = gen_case(fg, qmcpy, family, kind, d, alpha, ns, B, fit_its=FIT_ITS.get(name, 3))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("wrote", name, "loss=%.10e" % float(out["loss"]), "fit loss", out["fit_loss_hist"])


if __name__ == "__main__":
    main()
