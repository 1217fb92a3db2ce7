"""GPU parity of fits with the adaptive nugget (adaptive_nugget=True: _FastInverseLogDetCache.__call__,
util.py:286-290 -- lams[l, l] += noise |tr_ll / tr_00|) against the REAL reference's fit trajectories
(tests/golden/make_golden_adaptive.py -> tests/golden/adaptive/*.npz).

One task: the ratio is tr_00 / tr_00 = 1 exactly, so the device-resident spectral fit (the plain nugget) runs; the
test checks that it does and matches the reference.  Multitask (T = 2, the learned task kernel): the ratio
|tr_11 / tr_00| scales the second task's nugget -- through the device-resident general multitask fit
(fgp_mt_fit_desc.nugget_coef, ABI 16: the ratio from the pair spectra's sums, its noise and lengthscale
derivatives in closed form) and through the generic autograd loop (FGP_MT_FUSED=0).
Tolerances as the golden fits (tests/test_gpu_gp.py): loss history 2e-7 relative, parameters 1e-10, post_mean
1e-8 relative, post_var 1e-8 K(x, x).
"""
import glob
import os

import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from tests.gpu_fixtures import DEV, rel_err

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)

ADIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "adaptive")
NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(ADIR, "*.npz")))


def build(g):
    fam, d, alpha = str(g["family"]), int(g["d"]), int(g["alpha"])
    ns = [int(v) for v in g["ns"]]
    T = len(ns)
    kw = dict(alpha=alpha, adaptive_nugget=True, noise=float(g["noise"]), device=DEV)
    if T > 1:
        kw["num_tasks"] = T
    if fam == "lattice":
        seqs = [F.Lattice(d, randomize="SHIFT", generating_vector=g["z"], shift=g["shifts"][l]) for l in range(T)]
        gp = F.FastGPLattice(seqs if T > 1 else seqs[0], **kw)
    else:
        seqs = [F.DigitalNetB2(d, randomize="DS", generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                               shift=g["shifts"][l].astype(np.uint64)) for l in range(T)]
        gp = F.FastGPDigitalNetB2(seqs if T > 1 else seqs[0], **kw)
    if T > 1:
        xs = gp.get_x_next(torch.tensor(ns))
        for l in range(T):
            assert np.array_equal(xs[l].cpu().numpy(), g["x_%d" % l])
        gp.add_y_next([torch.from_numpy(g["y_%d" % l]).to(DEV) for l in range(T)])
    else:
        x = gp.get_x_next(ns[0])
        assert np.array_equal(x.cpu().numpy(), g["x_0"])
        gp.add_y_next(torch.from_numpy(g["y_0"]).to(DEV))
    return gp


def _spy(monkeypatch):
    """Count the device engines the fits build (FusedMLL: single task; MtGeneralEngine: multitask)."""
    from fastgaussianprocesses_amd import fit_engine, multitask
    engines = []
    for cls in (fit_engine.FusedMLL, multitask.MtGeneralEngine):
        orig = cls.__init__

        def init(self, *a, _orig=orig, **k):
            engines.append(type(self).__name__)
            return _orig(self, *a, **k)
        monkeypatch.setattr(cls, "__init__", init)
    return engines


@pytest.mark.parametrize("path", ["device", "generic"])
@pytest.mark.parametrize("name", NAMES)
def test_adaptive_nugget_fit_matches_reference(name, path, monkeypatch):
    g = np.load(os.path.join(ADIR, name + ".npz"))
    T = len(g["ns"])
    if path == "generic" and T == 1:
        pytest.skip("one task: the plain nugget (device fit) -- no separate generic case")
    monkeypatch.setenv("FGP_MT_FUSED", "1" if path == "device" else "0")
    engines = _spy(monkeypatch)
    gp = build(g)
    its = len(g["fit_loss_hist"]) - 1
    data = gp.fit(iterations=its, store_hists=True, verbose=0, stop_crit_wait_iterations=its + 5)
    if path == "device":
        assert engines == (["FusedMLL"] if T == 1 else ["MtGeneralEngine"]), engines
    else:
        assert not engines, engines
    assert rel_err(data["loss_hist"], g["fit_loss_hist"]) <= 2e-7
    assert rel_err(gp.raw_lengthscales, g["fit_raw_lengthscales"]) <= 1e-10
    assert rel_err(data["lengthscales_hist"], g["fit_lengthscales_hist"]) <= 1e-10
    assert rel_err(gp.raw_scale, g["fit_raw_scale"]) <= 1e-10
    xt = torch.from_numpy(g["x_test"]).to(DEV)
    assert rel_err(gp.post_mean(xt), g["fit_pmean"]) <= 1e-8
    pv = gp.post_var(xt).cpu()
    kxx = float(np.abs(g["fit_pvar"]).max()) + float(torch.exp(gp.raw_scale.detach()).max())
    assert float((pv - torch.from_numpy(g["fit_pvar"])).abs().max()) <= 1e-8 * kxx


@pytest.mark.parametrize("family", ["lattice", "net"])
def test_multitask_adaptive_nugget_device_equals_generic(family, monkeypatch):
    """Three tasks of unequal n (the reference's multitask example sizes [64, 8, 256]), the task kernel learned, the
    adaptive nugget: the device fit (its first loss against a one-iteration MtGeneralEngine evaluation) and the
    generic autograd loop, 8 iterations each: loss histories 5e-7 relative, lengthscales / task factor / noise
    1e-9 (sign-driven Rprop)."""
    from fastgaussianprocesses_amd.multitask import MtGeneralEngine
    d, T, ns = 2, 3, [64, 8, 256]

    def make():
        if family == "lattice":
            gp = F.FastGPLattice(d, seed_for_seq=5, num_tasks=T, adaptive_nugget=True, noise=1e-4, device=DEV)
        else:
            gp = F.FastGPDigitalNetB2(d, seed_for_seq=5, num_tasks=T, adaptive_nugget=True, noise=1e-4, device=DEV)
        xs = gp.get_x_next(n=torch.tensor(ns))
        gp.add_y_next([torch.sin(3 * xs[l]).sum(1) * (1 + l) + torch.cos(7 * xs[l][:, 0]) for l in range(T)])
        return gp
    gp = make()
    assert gp._mt_general_ok()
    eng = MtGeneralEngine(gp, 0.1, 2)
    eng.run(0, 1, final_no_update=True)
    torch.cuda.synchronize()
    loss = float(eng.loss_hist[0, 0, 0])
    out = {}
    for path in ("device", "generic"):
        monkeypatch.setenv("FGP_MT_FUSED", "1" if path == "device" else "0")
        gpp = make()
        data = gpp.fit(iterations=8, store_hists=True, verbose=0, stop_crit_wait_iterations=20)
        out[path] = (data["loss_hist"], gpp.raw_lengthscales.detach().cpu().clone(),
                     gpp.raw_factor_task_kernel.detach().cpu().clone(), gpp.raw_noise.detach().cpu().clone())
    (la, sa, fa, na), (lb, sb, fb, nb) = out["device"], out["generic"]
    assert abs(float(-la[0]) - loss) <= 1e-12 * abs(loss)
    assert rel_err(la, lb) <= 5e-7, (la, lb)
    assert rel_err(sa, sb) <= 1e-9 and rel_err(fa, fb) <= 1e-9 and rel_err(na, nb) <= 1e-9
