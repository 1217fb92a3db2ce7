"""Single-task API beyond beta = 0 and a unit task kernel, against the REAL reference's values
(tests/golden/make_golden_single_extras.py -> tests/golden/single_extras.npz):

* FastGPLattice / FastGPDigitalNetB2 .kernel(x, z, beta0, beta1, c0, c1) with derivative multi-indices
  (abstract_gp.py:693-706 -> abstract_fast_gp.py:173-196): the parts with derivative orders on the device
  (fgp_mt_parts), combined as the reference's _kernel_from_parts;
* a single-task GP with noise_task_kernel = 2.5 (gram_matrix_tasks = 2.5: ev = (sqrt(n) lambda + noise) Kt,
  util.py:285-298; kmat = Kt K, abstract_gp.py:375): fit(iterations=3), post_mean, post_var -- routed to the
  multitask class with T = 1 (its device-resident fit with a fixed task kernel).
"""
import os

import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from tests.gpu_fixtures import DEV, rel_err

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "single_extras.npz"))


def _seq(pre):
    d = int(G[pre + "d"]) if (pre + "d") in G.files else int(G["ts_d"])
    if (pre + "C") in G.files:
        return F.DigitalNetB2(d, randomize="DS", generating_matrices=G[pre + "C"].astype(np.uint64), t=int(G[pre + "t"]),
                              shift=G[pre + "shift"].astype(np.uint64))
    return F.Lattice(d, randomize="SHIFT", generating_vector=G[pre + "z"], shift=G[pre + "shift"])


@pytest.mark.parametrize("case", [0, 1, 2])
def test_single_task_derivative_kernel_matches_reference(case):
    pre = "k%d_" % case
    d, alpha = int(G[pre + "d"]), int(G[pre + "alpha"])
    cls = F.FastGPLattice if str(G[pre + "family"]) == "lattice" else F.FastGPDigitalNetB2
    gp = cls(_seq(pre), alpha=alpha, scale=1.7, lengthscales=torch.tensor([0.6, 1.4, 0.9][:d]), device=DEV)
    assert type(gp) is cls                                       # the single-task class
    x = gp.get_x_next(16)
    assert np.array_equal(x.cpu().numpy(), G[pre + "x"])
    z = torch.from_numpy(G[pre + "z_test"]).to(DEV)
    b0, b1 = torch.from_numpy(G[pre + "beta0"]), torch.from_numpy(G[pre + "beta1"])
    c0, c1 = torch.from_numpy(G[pre + "c0"]), torch.from_numpy(G[pre + "c1"])
    k = gp.kernel(x[:, None, :], z[None, :, :], b0, b1, c0, c1)
    ref = G[pre + "kernel"]
    assert tuple(k.shape) == ref.shape
    assert rel_err(k, ref) <= 1e-12
    # beta = 0, unit coefficients: the same value as the plain kernel
    zero = torch.zeros((1, d), dtype=torch.int64)
    k0 = gp.kernel(x[:, None, :], z[None, :, :], zero, zero, torch.ones(1), torch.ones(1))
    assert rel_err(k0, gp.kernel(x[:, None, :], z[None, :, :])) <= 1e-13


def test_single_task_non_unit_task_kernel_matches_reference():
    m, d, its = int(G["ts_m"]), int(G["ts_d"]), int(G["ts_its"])
    gp = F.FastGPLattice(_seq("ts_"), alpha=2, noise_task_kernel=2.5, device=DEV)
    assert float(gp.gram_matrix_tasks.reshape(-1)[0]) == 2.5
    x = gp.get_x_next(2 ** m)
    assert np.array_equal(x.cpu().numpy(), G["ts_x"])
    gp.add_y_next(torch.from_numpy(G["ts_y"]).to(DEV))
    data = gp.fit(iterations=its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=its + 5)
    olh = torch.from_numpy(G["ts_loss_hist"])
    assert float((data["loss_hist"].cpu() - olh).abs().max()) <= 2e-7 * float(olh.abs().max())
    assert float((gp.raw_lengthscales.detach().cpu() - torch.from_numpy(G["ts_raw_lengthscales"])).abs().max()) <= 1e-10
    assert float((gp.raw_scale.detach().cpu() - torch.from_numpy(G["ts_raw_scale"])).abs().max()) <= 1e-10
    xt = torch.from_numpy(G["ts_x_test"]).to(DEV)
    pm = gp.post_mean(xt).cpu()
    assert pm.shape == G["ts_pmean"].shape
    assert rel_err(pm, G["ts_pmean"]) <= 1e-7
    pv = gp.post_var(xt).cpu()
    assert float((pv - torch.from_numpy(G["ts_pvar"])).abs().max()) <= 1e-8 * float(G["ts_kxx"])
