"""GPU parity of the PARAMETER-BATCHED multitask GP of docs/examples/batch_multitask/fgp_lattice.ipynb (cell 6:
shape_batch = [2, 3, 4], 5 tasks with n = 2^[6, 5, 4, 3, 2], scale / lengthscales / noise / task factor / task noise
each with batch dimensions broadcast to shape_batch, abstract_gp.py:73-139) against the REAL reference
(tests/golden/make_golden_batch_mt.py -> tests/golden/batch_mt/*.npz): the lattice GP of the notebook (d = 6) and a
digital net of the same shapes (d = 3, alpha = 2).

The device-resident fit (fgp_mt_fit_run over G = 24 eigen-problems, ABI 16: every output its own problem, its
parameters the rows of each parameter block, a row shared by several outputs summing their gradients) and the
generic autograd loop (FGP_MT_FUSED=0) against the reference's 4-iteration trajectory: loss history 2e-7 relative (the
multitask golden tolerance), every fitted raw parameter 1e-9 (sign-driven Rprop: the trajectory is the reference's),
post_mean / post_var / post_cov after the fit 1e-8 relative / 1e-8 of the largest variance scale.
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

BDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "batch_mt")
NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(BDIR, "*.npz")))
PNAMES = ("raw_scale", "raw_lengthscales", "raw_noise", "raw_factor_task_kernel", "raw_noise_task_kernel")


def build(g):
    fam, d, alpha, T = str(g["family"]), int(g["d"]), int(g["alpha"]), int(g["T"])
    sb = [int(v) for v in g["shape_batch"]]
    kw = dict(alpha=alpha, num_tasks=T, shape_batch=sb, shape_scale=sb + [1], shape_lengthscales=sb[1:] + [d],
              shape_noise=sb[2:] + [1], shape_factor_task_kernel=sb + [T, T], shape_noise_task_kernel=sb[1:] + [T],
              device=DEV)
    if fam == "lattice":
        seqs = [F.Lattice(d, randomize="SHIFT", generating_vector=g["z"], shift=g["shifts"][l]) for l in range(T)]
        gp = F.FastGPLattice(seqs, **kw)
    else:
        seqs = [F.DigitalNetB2(d, randomize="DS", generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                               shift=g["shifts"][l].astype(np.uint64)) for l in range(T)]
        gp = F.FastGPDigitalNetB2(seqs, **kw)
    with torch.no_grad():
        for nm in PNAMES:
            p = getattr(gp, nm)
            assert tuple(p.shape) == tuple(g["init_" + nm].shape), nm
            p.copy_(torch.from_numpy(g["init_" + nm]).to(DEV))
    ns = [int(v) for v in g["ns"]]
    xs = gp.get_x_next(n=torch.tensor(ns))
    for l in range(T):
        assert np.array_equal(xs[l].cpu().numpy(), g["x_%d" % l])
    gp.add_y_next([torch.from_numpy(g["y_%d" % l]).to(DEV) for l in range(T)])
    return gp


@pytest.mark.parametrize("path", ["device", "generic"])
@pytest.mark.parametrize("name", NAMES)
def test_parameter_batched_multitask_fit_matches_reference(name, path, monkeypatch):
    g = np.load(os.path.join(BDIR, name + ".npz"))
    monkeypatch.setenv("FGP_MT_FUSED", "1" if path == "device" else "0")
    gp = build(g)
    if path == "device":
        assert gp._mt_general_ok(), "the notebook's parameter batch runs the device-resident fit"
        assert gp._mt_param_rows() is not None
    its = len(g["fit_loss_hist"]) - 1
    data = gp.fit(iterations=its, store_hists=True, verbose=0, stop_crit_wait_iterations=its + 5)
    assert rel_err(data["loss_hist"], g["fit_loss_hist"]) <= 2e-7, (data["loss_hist"], g["fit_loss_hist"])
    for nm in PNAMES:
        assert float((getattr(gp, nm).detach().cpu() - torch.from_numpy(g["fit_" + nm])).abs().max()) <= 1e-9, nm
    xt = torch.from_numpy(g["x_test"]).to(DEV)
    assert rel_err(gp.post_mean(xt), g["fit_pmean"]) <= 1e-8
    pv = gp.post_var(xt).cpu()
    assert float((pv - torch.from_numpy(g["fit_pvar"])).abs().max()) <= 1e-8 * max(1.0, float(np.abs(g["fit_pvar"]).max()))
    pc = gp.post_cov(xt[:4], xt[4:9]).cpu()
    assert tuple(pc.shape) == g["fit_pcov"].shape          # shape_batch + [T, T, 4, 5]
    assert float((pc - torch.from_numpy(g["fit_pcov"])).abs().max()) <= 1e-8 * max(1.0, float(np.abs(g["fit_pcov"]).max()))


@pytest.mark.parametrize("name", NAMES)
def test_parameter_batched_multitask_loss_and_gradient(name, monkeypatch):
    """One device evaluation (MtGeneralEngine: fgp_mt_fit_run, no update) at the initial parameters: the summed MLL
    and the gradient of every learned raw parameter against the reference's autograd (2e-7 relative)."""
    from fastgaussianprocesses_amd.multitask import MtGeneralEngine
    g = np.load(os.path.join(BDIR, name + ".npz"))
    gp = build(g)
    eng = MtGeneralEngine(gp, 0.1, 2)
    assert eng.G == int(np.prod(g["shape_batch"]))
    eng.run(0, 1, final_no_update=True)
    torch.cuda.synchronize()
    assert abs(float(eng.loss_hist[0, 0, 0]) - float(g["loss"])) <= 2e-7 * abs(float(g["loss"]))
    grad = eng.grad.cpu()
    o = 0
    for nm, size in zip(PNAMES, eng.sizes):
        gv = grad[o:o + size]
        o += size
        if "grad_" + nm in g.files:
            ref = torch.from_numpy(g["grad_" + nm]).reshape(-1)
            assert rel_err(gv, ref) <= 2e-7, (nm, gv[:4], ref[:4])


def _general_fit_rows(gp, mode, its=6):
    """fit rows (loss history, raw parameter history) of the general device fit with the per-class kernel forced
    (fgp_set_mt_class_kernel: 1 thread per class, 2 wave per class)."""
    from fastgaussianprocesses_amd import _native as N
    from fastgaussianprocesses_amd.multitask import MtGeneralEngine
    N.call("fgp_set_mt_class_kernel", mode)
    try:
        eng = MtGeneralEngine(gp, 0.1, its + 1)
        eng.run(0, its + 1, final_no_update=True)
        torch.cuda.synchronize()
        return eng.loss_hist[:its + 1].cpu(), eng.raw_hist[:its + 1].cpu()
    finally:
        N.call("fgp_set_mt_class_kernel", 0)


@pytest.mark.parametrize("name", NAMES + ["mt:" + nm for nm in ("mt_lattice_d1_a2_T3", "mt_net_d2_a2_T3",
                                                                 "mt_lattice_d2_a2_T2_b2", "deriv_lattice_d2_a2")])
def test_wave_per_class_kernel_equals_thread_per_class(name, monkeypatch):
    """k_mtg_class (a wave per frequency class, the class in LDS) against k_mtg_factor_grad (a thread per class,
    the generic path's bodies): the whole fit trajectory bit for bit, on the parameter batch and on the
    unbatched multitask fixtures."""
    monkeypatch.setenv("FGP_MT_GENERAL", "1")
    if name.startswith("mt:"):
        from tests.golden_util import load_golden
        from tests.test_gpu_multitask import product_mt
        gp = product_mt(load_golden(name[3:]))
    else:
        gp = build(np.load(os.path.join(BDIR, name + ".npz")))
    la, ra = _general_fit_rows(gp, 1)
    lb, rb = _general_fit_rows(gp, 2)
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb) and torch.equal(ra, rb)
