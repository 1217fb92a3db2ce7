"""Batched hyper-parameter fits of independent fast GPs (e.g. the randomly shifted replicas of one
lattice GP, BASELINE config C4) in ONE device-resident loop.

fastgps fits each GP on its own (AbstractGP.fit, fastgps/abstract_gp.py:152-306).  On MI355X a single
n = 2^20 GP fills only 256 workgroups per pass, so independent GPs of the same family / n / d are
stacked into one fgp_fit_run with G problems (per_problem mode: every GP keeps its own loss, its own
Rprop state and its own early-stopping decision).  The result for each GP is exactly what its own
`gp.fit(...)` returns: the stopping rule is applied per GP on its own loss history, and each GP's
best parameters are restored (extra iterations run for GPs that stopped earlier are discarded).
"""
import math

import torch

from .fit_engine import FusedMLL, LatticePartsGen, mll_constant


def fit_batched(gps, iterations=5000, lr=None, stop_crit_improvement_threshold=5e-2, stop_crit_wait_iterations=10,
                store_hists=False, store_loss_hist=False):
    """Fit independent single-problem GPs (same class, n, d, alpha, shapes) with the fused MLL loop.

    Returns the list of per-GP `data` dicts that `gp.fit(iterations=..., verbose=0, ...)` would return."""
    assert len(gps) > 0
    g0 = gps[0]
    n = int(g0.n[0])
    for gp in gps:
        assert type(gp) is type(g0), "fit_batched needs GPs of one family"
        assert int(gp.n[0]) == n and gp.d == g0.d and gp._alphas == g0._alphas
        assert gp._fused_ok(), "every GP must qualify for the fused MLL path"
        assert gp._problem_batch()[1] == 1, "per-output hyper-parameters: fit those GPs individually"
        assert gp.raw_lengthscales.shape == g0.raw_lengthscales.shape
        assert (gp.raw_scale.requires_grad, gp.raw_lengthscales.requires_grad, gp.raw_noise.requires_grad) == \
               (g0.raw_scale.requires_grad, g0.raw_lengthscales.requires_grad, g0.raw_noise.requires_grad)
    eng = batched_engine(gps, iterations, lr)
    dev = g0.device
    dl = g0.raw_lengthscales.shape[-1]
    logtol = math.log(1 + stop_crit_improvement_threshold)
    state = [dict(best=math.inf, save=math.inf, waited=0, best_i=0, stop=None, losses=[]) for _ in gps]
    total = iterations + 1
    i0, chunk = 0, 4
    while any(s["stop"] is None for s in state) and i0 < total:
        k = min(chunk, total - i0)
        eng.run(i0, k, final_no_update=(i0 + k == total))
        lh = eng.loss_hist[i0:i0 + k, :, 0].cpu()
        for p, s in enumerate(state):
            if s["stop"] is not None:
                continue
            for r in range(k):
                i = i0 + r
                lv = float(lh[r, p])
                s["losses"].append(lv)
                if lv < s["best"]:
                    s["best"], s["best_i"] = lv, i
                if (s["save"] - lv) > logtol:
                    s["waited"] = 0
                    s["save"] = s["best"]
                else:
                    s["waited"] += 1
                if i == iterations or s["waited"] == stop_crit_wait_iterations:
                    s["stop"] = i
                    break
        i0 += k
        chunk = min(64, chunk * 2)
    S, L, _ = eng.sizes
    out = []
    best_rows = eng.raw_hist[torch.tensor([s["best_i"] for s in state], device=dev)]
    for p, (gp, s) in enumerate(zip(gps, state)):
        row = best_rows[p]
        with torch.no_grad():
            vals = {"raw_scale": row[p:p + 1], "raw_lengthscales": row[S + p * dl:S + (p + 1) * dl],
                    "raw_noise": row[S + L + p:S + L + p + 1]}
            for name, v in vals.items():
                old = getattr(gp, name)
                setattr(gp, name, torch.nn.Parameter(v.reshape(old.shape).clone(), requires_grad=old.requires_grad))
        gp._cache = {}
        gp._snap = None
        data = {"iterations": s["stop"]}
        if store_hists or store_loss_hist:
            data["loss_hist"] = torch.tensor([-v for v in s["losses"]])
        out.append(data)
    return out


def batched_engine(gps, iterations, lr=None):
    """The FusedMLL (per_problem mode) over the GPs' stacked problems: Y = |ytilde|^2 rows and raw
    parameters stacked, the kernel parts regenerated in the kernels for lattice GPs sharing one
    generating vector (otherwise a stacked [P, d, n] parts array)."""
    g0 = gps[0]
    n = int(g0.n[0])
    P = len(gps)
    d = g0.d
    dev = g0.device
    gens = [gp._parts_gen(n) for gp in gps]
    gen = None
    if all(g is not None for g in gens) and all(g.z == gens[0].z for g in gens):
        # lattice points regenerated in the kernels; only the P shifts (= x[0] rows) are stacked
        gen = LatticePartsGen(gens[0].z, gens[0].alphas, torch.cat([g.shift for g in gens], 0))
        parts = None
    else:
        parts = torch.empty((P, d, n), dtype=torch.float64, device=dev)
        for p, gp in enumerate(gps):
            gp._k1parts(n, out=parts[p])
    ysq = torch.stack([gp._ysq(*gp._problem_batch())[0] for gp in gps])
    d_out = int(torch.tensor(g0.shape_batch).prod())
    dl = g0.raw_lengthscales.shape[-1]
    return FusedMLL(g0._FAMILY, parts, ysq,
                    torch.stack([gp.raw_scale.detach().reshape(-1)[0] for gp in gps]),
                    torch.stack([gp.raw_lengthscales.detach().reshape(dl) for gp in gps]),
                    torch.stack([gp.raw_noise.detach().reshape(-1)[0] for gp in gps]),
                    logdet_weight=float(d_out), mll_const=mll_constant(d_out, n),
                    requires_grad=(g0.raw_scale.requires_grad, g0.raw_lengthscales.requires_grad,
                                   g0.raw_noise.requires_grad),
                    lr=1e-1 if lr is None else lr, max_iters=min(iterations + 1, 64), parts_per_problem=True,
                    per_problem=True, gen=gen)
