"""Generate golden input/output vectors from the REAL reference (fastgps @ /root/reference).

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [fixture names...]

The reference is imported through oracle/refshim/load_reference.py (in-memory PEP-646 rewrite +
qmcpy stand-in).  All point sets are EXPLICIT (generating vector / matrices + shift are
stored in each fixture) because qmcpy's defaults are unavailable offline.  Every fixture holds only
data: inputs and the reference's outputs.

What each fixture pins (reference file:line):
  ft_*/ift_*        AbstractFastGP.ft/ift (abstract_fast_gp.py:197-228) over qmcpy transforms
  k1parts, k1, lam  _K1PartsSeq (util.py:50-62), _kernel_from_parts (abstract_fast_gp.py:181-191),
                    _LamCaches (util.py:95-132)
  ytilde            _YtildeCache (util.py:168-183)
  logdet, norm_term _FastInverseLogDetCache (util.py:275-337,364-370)
  loss, grad_*      AbstractGP.fit MLL assembly (abstract_gp.py:235,253-260) + autograd (:294)
  coeffs            _CoeffsCache (util.py:419-425)
  pmean/pvar/pcov   post_mean/post_var/post_cov (abstract_gp.py:352-474)
  pcmean/pcvar      post_cubature_mean/var (abstract_fast_gp.py:65-109)
  fit_*             fit(iterations=3, store_hists=True) trajectory (abstract_gp.py:152-306)
  pvar_2n/pcvar_2n  projections with n=2n (abstract_fast_gp.py:41-46,82-109)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.refshim.load_reference import import_reference  # noqa: E402

# A rank-1 lattice generating vector for n up to 2^20 (odd entries; quality is not relied upon).
LATTICE_Z = [1, 182667, 469891, 498753, 110745, 446247, 250185, 118627, 245333, 283199]

# Joe-Kuo style Sobol' initial direction numbers (s, a, m_1..m_s) for dims 2..8; dim 1 = identity.
_SOBOL_INIT = [
    (1, 0, [1]),
    (2, 1, [1, 3]),
    (3, 1, [1, 3, 1]),
    (3, 2, [1, 1, 1]),
    (4, 1, [1, 1, 3, 3]),
    (4, 4, [1, 3, 5, 13]),
    (5, 2, [1, 1, 5, 5, 17]),
]


def sobol_generating_matrices(d, t=32, mmax=32):
    """Columns of the t x mmax generating matrices as t-bit ints (MSB = first binary digit)."""
    C = np.zeros((d, mmax), dtype=np.uint64)
    for k in range(mmax):
        C[0, k] = np.uint64(1) << np.uint64(t - 1 - k)
    for j in range(1, d):
        s, a, minit = _SOBOL_INIT[j - 1]
        m = list(minit)
        for k in range(s, mmax):
            new = m[k - s] ^ (m[k - s] << s)
            for q in range(1, s):
                if (a >> (s - 1 - q)) & 1:
                    new ^= m[k - q] << q
            m.append(new)
        for k in range(mmax):
            # direction number v_k = m_k / 2^(k+1) -> t-bit integer
            C[j, k] = np.uint64(m[k]) << np.uint64(t - 1 - k)
    return C


def f_ackley(x, a=20, b=0.2, c=2 * np.pi, scaling=32.768):
    # the reference's doctest workload (fast_gp_lattice.py:14-22)
    x = 2 * scaling * x - scaling
    t1 = a * torch.exp(-b * torch.sqrt(torch.mean(x ** 2, 1)))
    t2 = torch.exp(torch.mean(torch.cos(c * x), 1))
    return -t1 - t2 + a + np.exp(1)


def make_y(x, B):
    f = f_ackley(x)
    if B == 0:
        return f
    return torch.stack([f * (1 + 0.1 * b) + 0.01 * b * torch.cos(2 * np.pi * x[:, 0]) for b in range(B)], 0)


def _np(t):
    t = t.detach()
    return t.cpu().numpy() if t.is_complex() or t.dtype != torch.bfloat16 else t.float().numpy()


def gen_case(fg, qmcpy, family, m, d, alpha, B=0, per_output=False, seed=7, fit_its=3):
    n = 2 ** m
    out = {"family": np.array(family), "m": np.array(m), "d": np.array(d), "alpha": np.array(alpha),
           "B": np.array(B), "per_output": np.array(per_output)}
    shape_batch = [B] if B > 0 else []
    kw = dict(alpha=alpha, shape_batch=shape_batch)
    if per_output:
        kw["shape_scale"] = [B, 1]
        kw["shape_lengthscales"] = [B, d]
    if family == "lattice":
        shift = np.random.default_rng(seed).uniform(size=d)
        seq = qmcpy.Lattice(d, randomize="SHIFT", generating_vector=LATTICE_Z[:d], shift=shift)
        out["z"] = np.array(LATTICE_Z[:d], dtype=np.int64)
        out["shift"] = shift
        fgp = fg.FastGPLattice(seq, **kw)
    else:
        t = 32
        C = sobol_generating_matrices(d, t=t)
        shift = np.random.default_rng(seed).integers(0, 2 ** t, size=d, dtype=np.uint64)
        seq = qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=C, t=t, shift=shift)
        out["C"] = C.astype(np.int64)
        out["t"] = np.array(t)
        out["shift"] = shift.astype(np.int64)
        fgp = fg.FastGPDigitalNetB2(seq, **kw)
    x = fgp.get_x_next(n)
    y = make_y(x, B)
    fgp.add_y_next(y)
    out["x"] = _np(x)
    out["xb"] = _np(fgp.get_xb(0))
    out["y"] = _np(y)
    # raw transforms (stabilised wrappers) on seeded inputs
    g = torch.Generator().manual_seed(100 + m)
    ft_in = torch.randn((3, n), generator=g) + 5.0
    out["ft_in"] = _np(ft_in)
    out["ft_out"] = _np(fgp.ft(ft_in))
    if family == "lattice":
        ift_in = torch.randn((3, n), generator=g) + 1j * torch.randn((3, n), generator=g)
    else:
        ift_in = torch.randn((3, n), generator=g)
    out["ift_in"] = _np(ift_in)
    out["ift_out"] = _np(fgp.ift(ift_in))
    # caches at initial hyperparameters
    out["k1parts"] = _np(fgp.get_k1parts(0, 0))
    lam = fgp.get_lam(0, 0)
    out["lam"] = _np(lam)
    out["ytilde"] = _np(fgp.get_ytilde(0))
    # MLL + autograd gradient exactly as fit() forms it (abstract_gp.py:235,253-260,294)
    os.environ["FASTGP_FORCE_RECOMPILE"] = "True"
    cache = fgp.get_inv_log_det_cache()
    norm_term, logdet = cache.get_norm_term_logdet_term()
    d_out = int(torch.tensor(fgp.shape_batch).prod())
    mll_const = d_out * fgp.n.sum() * np.log(2 * np.pi)
    term1 = norm_term.sum()
    term2 = d_out / torch.tensor(logdet.shape).prod() * logdet.sum()
    loss = 0.5 * (term1 + term2 + mll_const)
    gs, gl = torch.autograd.grad(loss, [fgp.raw_scale, fgp.raw_lengthscales])
    del os.environ["FASTGP_FORCE_RECOMPILE"]
    out["norm_term"] = _np(norm_term)
    out["logdet"] = _np(logdet)
    out["loss"] = _np(loss)
    out["grad_raw_scale"] = _np(gs)
    out["grad_raw_lengthscales"] = _np(gl)
    # predictions
    gt = torch.Generator().manual_seed(17)
    xt = torch.rand((16, d), generator=gt)
    out["x_test"] = _np(xt)
    out["coeffs"] = _np(fgp.coeffs)
    out["pmean"] = _np(fgp.post_mean(xt))
    out["pvar"] = _np(fgp.post_var(xt))
    out["pcov"] = _np(fgp.post_cov(xt[:4], xt[4:9]))
    out["pcmean"] = _np(fgp.post_cubature_mean())
    out["pcvar"] = _np(fgp.post_cubature_var())
    out["pvar_2n"] = _np(fgp.post_var(xt, n=2 * n))
    out["pcvar_2n"] = _np(fgp.post_cubature_var(n=2 * n))
    # fit trajectory
    data = fgp.fit(iterations=fit_its, store_hists=True, verbose=0, stop_crit_wait_iterations=fit_its + 5)
    out["fit_iterations"] = np.array(data["iterations"])
    out["fit_loss_hist"] = _np(data["loss_hist"])
    out["fit_scale_hist"] = _np(data["scale_hist"])
    out["fit_lengthscales_hist"] = _np(data["lengthscales_hist"])
    out["fit_raw_scale"] = _np(fgp.raw_scale)
    out["fit_raw_lengthscales"] = _np(fgp.raw_lengthscales)
    out["fit_pmean"] = _np(fgp.post_mean(xt))
    out["fit_pvar"] = _np(fgp.post_var(xt))
    return out


CASES = [
    # family, m, d, alpha, B, per_output
    ("lattice", 0, 1, 2, 0, False),
    ("lattice", 1, 1, 2, 0, False),
    ("lattice", 4, 1, 1, 0, False),
    ("lattice", 4, 3, 2, 0, False),
    ("lattice", 6, 2, 3, 0, False),
    ("lattice", 7, 3, 4, 0, False),
    ("lattice", 10, 3, 2, 0, False),
    ("lattice", 12, 5, 2, 0, False),
    ("lattice", 13, 2, 2, 0, False),
    ("lattice", 10, 2, 2, 3, False),
    ("lattice", 9, 2, 2, 3, True),
    ("net", 1, 1, 1, 0, False),
    ("net", 4, 1, 1, 0, False),
    ("net", 4, 3, 1, 0, False),
    ("net", 10, 3, 1, 0, False),
    ("net", 12, 5, 1, 0, False),
    ("net", 13, 2, 1, 0, False),
    ("net", 10, 2, 1, 3, False),
    # Walsh orders 2-4 (the reference's default alpha = 2): the reference's pipeline with qmcpy's
    # weighted_walsh_funcs restated by the stand-in (parity at that boundary unpinned)
    ("net", 4, 2, 2, 0, False),
    ("net", 10, 3, 2, 0, False),
    ("net", 11, 2, 3, 0, False),
    ("net", 9, 3, 4, 0, False),
    ("net", 10, 2, 2, 3, False),
]


def case_name(c):
    family, m, d, alpha, B, po = c
    return "%s_m%d_d%d_a%d_b%d%s" % (family, m, d, alpha, B, "_po" if po else "")


def main():
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    only = set(sys.argv[1:])          # optional: regenerate only the named fixtures
    for c in CASES:
        name = case_name(c)
        if only and name not in only:
            continue
        out = gen_case(fg, qmcpy, *c)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("wrote", name, "loss=%.10e" % float(out["loss"]))


if __name__ == "__main__":
    main()
