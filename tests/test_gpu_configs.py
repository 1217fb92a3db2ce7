"""Parity at the BASELINE.json configurations (C2: FastGPLattice n=2^16 d=3; C3: FastGPDigitalNetB2
n=2^16 d=3 with the reference's default alpha=2; C4: FastGPLattice n=2^20 d=5, the bench workload):
the drop-in classes on the GPU (fused fit kernels, matrix-free post_mean, Parseval post_var) against
the CPU oracle (oracle/fgp_oracle.py, the reference's op sequence in torch-CPU) on the same points and
data.  Tolerances as tests/test_gpu_gp.py: MLL trajectory 2e-7 relative (ill-conditioned at the
nugget), posterior mean 1e-7 relative, posterior variance 1e-8 K(x,x) absolute.
"""
import pytest
import torch

import fastgaussianprocesses_amd as F
from oracle import fgp_oracle as O
from tests.gpu_fixtures import DEV

pytestmark = pytest.mark.gpu
torch.set_default_dtype(torch.float64)


@pytest.mark.parametrize("family,m,d,its,npm,npv", [("lattice", 16, 3, 5, 32, 4), ("net", 16, 3, 5, 32, 4),
                                                    ("lattice", 20, 5, 3, 8, 2)])
def test_config_fit_and_predict_match_oracle(family, m, d, its, npm, npv):
    n = 2 ** m
    if family == "lattice":
        gp = F.FastGPLattice(F.Lattice(d, seed=7), device=DEV)
    else:
        gp = F.FastGPDigitalNetB2(F.DigitalNetB2(d, seed=7), device=DEV)   # default alpha = 2
    x = gp.get_x_next(n)
    y = O.f_ackley(x.cpu())
    gp.add_y_next(y.to(DEV))
    data = gp.fit(iterations=its, store_hists=True, verbose=0, stop_crit_wait_iterations=its + 5)
    o = O.OracleFastGP(family, x.cpu(), gp.get_xb().cpu() if family == "net" else None, y,
                       alpha=gp._alphas[0], t=getattr(gp, "t", None))
    od = o.fit(iterations=its, stop_crit_wait_iterations=its + 5)
    lh, olh = data["loss_hist"], od["loss_hist"]
    assert float((lh - olh).abs().max()) <= 2e-7 * float(olh.abs().max())
    assert float((gp.raw_lengthscales.detach().cpu() - o.raw_lengthscales.detach()).abs().max()) <= 1e-10
    xt = torch.rand((npm, d), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt.to(DEV)).cpu()
    opm = o.post_mean(xt)
    assert float((pm - opm).abs().max()) <= 1e-7 * float(opm.abs().max())
    pv = gp.post_var(xt[:npv].to(DEV)).cpu()
    opv = o.post_var(xt[:npv])
    kxx = float(o.kernel(xt[:npv], xt[:npv]).detach().abs().max())
    assert float((pv - opv.detach()).abs().max()) <= 1e-8 * kxx
