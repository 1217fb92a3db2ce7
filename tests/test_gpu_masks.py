"""fit(masks=...) (abstract_gp.py:152-306: only the outputs y[..., *masks] enter the MLL; d_out, the MLL constant and the
logdet term count the selected outputs) on the device: with hyper-parameters shared by the outputs, the fused fit runs
on Y = sum over the selected outputs of |ytilde_b|^2 (FastGP._masked_ysq); against the REAL reference's trajectories
(tests/golden/make_golden_masks.py -> tests/golden/masks/*.npz) and against the generic autograd loop.  Tolerances of
tests/test_gpu_gp.py: loss history 2e-7 relative, lengthscale trajectory 1e-10, post_mean 1e-7."""
import glob
import os

import numpy as np
import pytest
import torch

from tests.gpu_fixtures import product_gp, rel_err
from tests.golden_util import load_golden

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)

MASK_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "masks")
NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(MASK_DIR, "*.npz")))


@pytest.mark.parametrize("name", NAMES)
def test_masked_fit_matches_reference_on_device(name, monkeypatch):
    from fastgaussianprocesses_amd import fit_engine
    with np.load(os.path.join(MASK_DIR, name + ".npz"), allow_pickle=False) as f:
        g = {k: f[k] for k in f.files}
    src = load_golden(str(g["source"]))
    out = {}
    for path in ("device", "generic"):
        calls = []
        orig = fit_engine.FusedMLL.__init__

        def init(self, *a, **k):
            calls.append(1)
            return orig(self, *a, **k)
        monkeypatch.setattr(fit_engine.FusedMLL, "__init__", init)
        gp = product_gp(src)
        if path == "generic":
            monkeypatch.setattr(type(gp), "_masked_ysq", lambda self, masks: None)
        its = len(g["loss_hist"]) - 1
        data = gp.fit(iterations=its, store_hists=True, verbose=0, stop_crit_wait_iterations=its + 5,
                      masks=torch.from_numpy(g["mask"]))
        assert bool(calls) == (path == "device"), (path, calls)
        assert rel_err(data["loss_hist"], g["loss_hist"]) <= 2e-7
        assert rel_err(data["lengthscales_hist"], g["lengthscales_hist"]) <= 1e-10
        assert rel_err(gp.raw_lengthscales, g["raw_lengthscales"]) <= 1e-10
        xt = torch.from_numpy(src["x_test"]).to(gp.device)
        assert rel_err(gp.post_mean(xt), g["pmean"]) <= 1e-7
        out[path] = data["loss_hist"]
        monkeypatch.undo()
    assert rel_err(out["device"], out["generic"]) <= 2e-7
