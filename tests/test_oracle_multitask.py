"""Pin the multitask / derivative-informed oracle (oracle/fgp_oracle_mt.py) against golden vectors made
by the REAL reference (tests/golden/make_golden_multitask.py).  CPU only."""
import numpy as np
import pytest
import torch

from golden_util import golden_names, load_golden
from oracle.fgp_oracle_mt import OracleMultiTaskFastGP

torch.set_default_dtype(torch.float64)

MT_NAMES = golden_names(multitask=True)

# Fixtures where the REFERENCE's own block inverse is inaccurate, with the relative error it carries.
# deriv_lattice_d2_a3_equal: (f, df/dx0, df/dx1), alpha = 3, n = 128 each.  At frequency classes 12 and
# 116 the f-f eigenvalue is 1e-4 of the derivative block (eigenvalues 1.1e-4, 0.14, 1.0e4); the
# reference's unpivoted complex Schur recursion (util.py:301-323) pivots on it and its complement S
# comes out as 0.0049 - 0.0039i, where a Hermitian matrix's Schur complement is real.  Its logdet is
# -1381.633 against -1382.114 from slogdet, eigvalsh and Cholesky of the very same lams blocks (all
# three agree to 1e-10; tests/golden/check_mt_reference_logdet.py reproduces this).  Quantities that go through the
# inverse are therefore compared at that error; everything before the inverse (parts, lam, ytilde)
# at the usual tolerances.
REF_INVERSE_ERROR = {"deriv_lattice_d2_a3_equal": 2e-2}

# Prediction tolerances of fixtures whose posterior quantities are ill-conditioned (defaults in the tests).
# deriv_lattice_d2_a2_equal: (f, df/dx0, df/dx1), alpha = 2, n = 256 per task.  The oracle's dense inverse
# and the reference's block recursion agree to 4.3e-10 (inv), 1.4e-10 (coeffs), 1.4e-11 (loss) and the
# 8-iteration fit trajectory exactly, but sums of O(1e3) derivative-kernel values against that inverse
# cancel: post_mean differs by 2.7e-6 relative, post_var by 9e-8 kxx, post_cov by 4e-4 kxx, and the
# projection to n_new = [1024, 512, 2048] (blocks of cond ~1e12) by 69 % -- not a quantity fp64 pins, so
# it is not compared.  Measured in this container (oracle vs the reference's own values).
# deriv_lattice_d2_a2_equal_n1024: the same at n = 1024 per task (the probnum25 paper's size), conditioning
# ~1e8 worse: inv agrees to 3.6e-7, logdet to 3.6e-8, loss / gradients to 1e-7 and the 12-iteration fit
# trajectory exactly, but every posterior quantity of the fitted or initial GP moves by 10 % .. 100 %
# between two correct fp64 inverses (post_mean 12 %, post_cov 170 kxx): only the fit is compared.
PRED_TOL = {"deriv_lattice_d2_a2_equal": dict(pmean=1e-5, pvar=1e-6, pcov=2e-3, pvar_new=None, fit_pmean=1e-5),
            "deriv_lattice_d2_a2_equal_n1024": dict(logdet=1e-7, predictions=False)}


def pred_tol(name, key, default):
    return PRED_TOL.get(name, {}).get(key, default)



def make_oracle(g):
    fam = str(g["family"])
    T = len(g["ns"])
    ys = [torch.from_numpy(g["y_%d" % l]) for l in range(T)]
    derivs = None
    if str(g["kind"]) == "deriv":
        derivs = [torch.from_numpy(v) for v in g["derivatives"]]
    if fam == "lattice":
        return OracleMultiTaskFastGP("lattice", g["z"], g["shifts"], ys, alpha=int(g["alpha"]), derivatives=derivs)
    return OracleMultiTaskFastGP("net", g["C"], g["shifts"], ys, alpha=int(g["alpha"]), t=int(g["t"]),
                                 derivatives=derivs)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


@pytest.mark.parametrize("name", MT_NAMES)
def test_multitask_oracle_matches_reference(name):
    g = load_golden(name)
    o = make_oracle(g)
    T = o.T
    for l in range(T):
        x, xb = o.points(l, int(g["ns"][l]))
        assert np.array_equal(x.numpy(), g["x_%d" % l])
        assert np.array_equal(xb.numpy(), g["xb_%d" % l])
    for a in range(T):
        for b in range(a, T):
            n = max(int(g["ns"][a]), int(g["ns"][b]))
            kp = o.k1parts(a, b, n)
            assert rel(kp.numpy(), g["k1parts_%d%d" % (a, b)]) < 1e-13
            assert rel(o.lam(a, b, n).detach().numpy(), g["lam_%d%d" % (a, b)]) < 1e-12
        assert rel(o.ytilde(a).numpy(), g["ytilde_%d" % a]) < 1e-12
    assert rel(o.gram_matrix_tasks.detach().numpy(), g["gram_matrix_tasks"]) == 0.0
    tol = REF_INVERSE_ERROR.get(name)
    if tol is not None:
        loss = o.mll_loss()
        assert abs(loss.item() - float(g["loss"])) <= tol * abs(float(g["loss"]))
        # the reference's coefficients inherit the error: its post_mean is O(1e5) where the data are
        # O(1).  The oracle is held to the reference's own doctest criterion instead -- the posterior
        # mean interpolates the data at the training points (fast_gp_lattice.py:40, atol 1e-3).
        xt = torch.from_numpy(g["x_test"])
        for l in range(T):
            xl, _ = o.points(l, int(g["ns"][l]))
            assert float((o.post_mean(xl)[l] - o.ys[l]).abs().max()) < 1e-3
        assert rel(g["pmean"], o.post_mean(xt).numpy()) > 1e3      # documents the reference's failure
        return
    A, logdet, to, nsrt, nmin = o.inv_logdet()
    inv_ref = g["inv"]
    assert A.shape == inv_ref.shape
    assert rel(A.detach().numpy() if np.iscomplexobj(inv_ref) else A.detach().real.numpy(), inv_ref) < 1e-6
    assert abs(float(logdet.detach()) - float(g["logdet"].reshape(-1)[0])) <= \
        pred_tol(name, "logdet", 1e-8) * abs(float(g["logdet"].reshape(-1)[0])) + 1e-8
    norm, _ = o.norm_logdet()
    assert rel(norm.detach().numpy().reshape(-1), g["norm_term"].reshape(-1)) < 1e-7
    loss = o.mll_loss()
    assert abs(loss.item() - float(g["loss"])) <= 2e-7 * abs(float(g["loss"]))
    params = dict(raw_scale=o.raw_scale, raw_lengthscales=o.raw_lengthscales, raw_noise=o.raw_noise,
                  raw_factor_task_kernel=o.raw_factor_task_kernel, raw_noise_task_kernel=o.raw_noise_task_kernel)
    names = [str(s) for s in g["grad_names"]]
    grads = torch.autograd.grad(loss, [params[nm] for nm in names])
    for nm, gr in zip(names, grads):
        assert rel(gr.numpy(), g["grad_" + nm]) < 2e-6, nm
    xt = torch.from_numpy(g["x_test"])
    assert rel(o.coeffs().detach().numpy(), g["coeffs"]) < 1e-5
    if not pred_tol(name, "predictions", True):
        return
    assert rel(o.post_mean(xt).numpy(), g["pmean"]) < pred_tol(name, "pmean", 1e-7)
    kxx = max(float(o.scale), float(np.max(np.abs(g["pvar"]))), float(np.max(np.abs(g["pcvar"])))) * 10
    assert np.max(np.abs(o.post_var(xt).numpy() - g["pvar"])) <= pred_tol(name, "pvar", 1e-8) * kxx
    assert np.max(np.abs(o.post_cov(xt[:4], xt[4:9]).numpy() - g["pcov"])) <= pred_tol(name, "pcov", 1e-7) * kxx
    assert rel(o.post_cubature_mean().numpy(), g["pcmean"]) < 1e-8
    assert np.max(np.abs(o.post_cubature_var().numpy() - g["pcvar"])) <= 1e-8 * kxx
    assert np.max(np.abs(o.post_cubature_cov().numpy() - g["pccov"])) <= 1e-8 * kxx
    n_new = [int(v) for v in g["n_new"]]
    # post_var at the projected n: the blocks reach cond 4e8 at n = [256, 16, 2048] for the derivative
    # fixture (eigenvalues 1.9e-4 .. 8e4) and k(x,x) - k^T K^-1 k cancels O(1e3) kernel values down to
    # O(1); the reference's own value moves by 1.2 % there (ours is self-consistent: inv vs eigh-inverse
    # 2.7e-10), so the tolerance follows the conditioning of the fixture
    tol_new = 2e-2 * float(np.max(np.abs(g["pvar_new"]))) if str(g["kind"]) == "deriv" else 1e-8 * kxx
    if pred_tol(name, "pvar_new", 0.0) is not None:
        assert np.max(np.abs(o.post_var(xt, n_new).numpy() - g["pvar_new"])) <= tol_new
    assert np.max(np.abs(o.post_cubature_var(n_new).numpy() - g["pcvar_new"])) <= 1e-8 * kxx


@pytest.mark.parametrize("name", MT_NAMES)
def test_multitask_oracle_fit_trajectory(name):
    if name in REF_INVERSE_ERROR:
        pytest.skip("the reference's own inverse is inaccurate for this fixture (REF_INVERSE_ERROR)")
    g = load_golden(name)
    o = make_oracle(g)
    its = int(g["fit_iterations"])
    data = o.fit(iterations=its, stop_crit_wait_iterations=its + 5)
    assert data["iterations"] == its
    assert rel(data["loss_hist"].numpy(), g["fit_loss_hist"]) < 2e-7
    assert rel(data["lengthscales_hist"].numpy(), g["fit_lengthscales_hist"]) < 1e-10
    assert rel(data["scale_hist"].numpy(), g["fit_scale_hist"]) < 1e-10
    assert rel(data["task_kernel_hist"].numpy(), g["fit_task_kernel_hist"]) < 1e-10
    xt = torch.from_numpy(g["x_test"])
    if pred_tol(name, "predictions", True):
        assert rel(o.post_mean(xt).numpy(), g["fit_pmean"]) < pred_tol(name, "fit_pmean", 1e-7)
