"""Golden vectors for the BENCHED C2 / C3 work (BASELINE configs C2: FastGPLattice n = 2^16, d = 3; C3:
FastGPDigitalNetB2 n = 2^16, d = 3 with the reference's default alpha = 2) from the REAL reference, at the
length bench.py times them: fit(iterations=50, stop_crit_wait_iterations=51), then post_mean at 16 test points
and post_var at the first 2 (VERDICT r05 "Next round" item 1).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c23.py

The point sets are bench.SingleGP's: the package's Lattice(3, seed=7) (generating vector LATTICE_Z, shift
default_rng(7).uniform(size=3)) and DigitalNetB2(3, seed=7) (the Sobol' matrices of make_golden.py, t = 32,
digital shift default_rng(7).integers(0, 2^32, size=3)); y = f_ackley(x).

Writes tests/golden/c2_m16_d3_it50.npz, tests/golden/c3_m16_d3_a2_it50.npz (inputs: generating vector /
matrices, shift, test points; the reference's outputs: loss history, fitted raw parameters, post_mean,
post_var, K(x, x)) and profiles/r06_c23_backend_spread.json: the same runs with the reference's transform
replaced -- lattice: numpy's pocketfft (make_golden_c5's differentiable wrappers); net: a Walsh-Hadamard
butterfly with its stages in the opposite order and the 1/sqrt(2) applied per stage (a differentiable,
self-adjoint wrapper) -- the spread a correct implementation of the reference shows over these 50
iterations.  tests/test_gpu_bench_path.py allows 5x it.
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from oracle.refshim.load_reference import import_reference  # noqa: E402
from make_golden import LATTICE_Z, f_ackley, sobol_generating_matrices  # noqa: E402
from make_golden_c5 import _NpFFTBR, _NpIFFTBR, rel  # noqa: E402

M, D, ITS, NM, NV = 16, 3, 50, 16, 2


def _fwht_rev(x):
    """Orthonormal Sylvester-order WHT, stages from the widest butterfly down, 1/sqrt(2) per stage."""
    n = x.size(-1)
    shape = x.shape[:-1]
    y = x.clone()
    h = n // 2
    r = 1.0 / np.sqrt(2.0)
    while h >= 1:
        y = y.reshape(shape + (n // (2 * h), 2, h))
        a, b = y[..., 0, :], y[..., 1, :]
        y = torch.stack([(a + b) * r, (a - b) * r], dim=-2).reshape(shape + (n,))
        h //= 2
    return y


class _RevFWHT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _fwht_rev(x.detach()).clone()

    @staticmethod
    def backward(ctx, g):
        return _fwht_rev(g)


def run(fg, qmcpy, family):
    n = 2 ** M
    if family == "lattice":
        shift = np.random.default_rng(7).uniform(size=D)
        seq = qmcpy.Lattice(D, randomize="SHIFT", generating_vector=LATTICE_Z[:D], shift=shift)
        gp = fg.FastGPLattice(seq, alpha=2)
        inputs = dict(z=np.array(LATTICE_Z[:D], dtype=np.int64), shift=shift)
    else:
        t = 32
        C = sobol_generating_matrices(D, t=t)
        shift = np.random.default_rng(7).integers(0, 2 ** t, size=D, dtype=np.uint64)
        seq = qmcpy.DigitalNetB2(D, randomize="DS", generating_matrices=C, t=t, shift=shift)
        gp = fg.FastGPDigitalNetB2(seq, alpha=2)
        inputs = dict(C=C.astype(np.int64), t=np.array(t), shift=shift.astype(np.int64))
    x = gp.get_x_next(n)
    gp.add_y_next(f_ackley(x))
    t0 = time.perf_counter()
    data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=ITS + 1)
    t_fit = time.perf_counter() - t0
    xt = torch.rand((NM, D), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt)
    pv = gp.post_var(xt[:NV])
    out = dict(inputs, x_test=xt.numpy(), loss_hist=data["loss_hist"].detach().numpy(),
               raw_scale=gp.raw_scale.detach().numpy().reshape(-1),
               raw_lengthscales=gp.raw_lengthscales.detach().numpy().reshape(-1),
               pmean=pm.detach().numpy(), pvar=pv.detach().numpy(),
               kxx=gp.kernel(xt[:NV], xt[:NV]).detach().numpy().reshape(-1).real)
    print("%s: fit %.2f s (%.1f ms/it), final loss %.8f" % (family, t_fit, 1e3 * t_fit / (ITS + 1),
                                                          float(out["loss_hist"][-1])), flush=True)
    return out


def main():
    torch.set_default_dtype(torch.float64)
    torch.set_num_threads(os.cpu_count() or 1)
    fg = import_reference()
    import qmcpy
    keep = (qmcpy.fftbr_torch, qmcpy.ifftbr_torch, qmcpy.fwht_torch)
    spread = {}
    for family, name in (("lattice", "c2_m16_d3_it50"), ("net", "c3_m16_d3_a2_it50")):
        ref = run(fg, qmcpy, family)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), m=np.array(M), d=np.array(D), its=np.array(ITS),
                            family=np.array(family), **{k: np.asarray(v) for k, v in ref.items()})
        if family == "lattice":
            qmcpy.fftbr_torch, qmcpy.ifftbr_torch = _NpFFTBR.apply, _NpIFFTBR.apply
        else:
            qmcpy.fwht_torch = _RevFWHT.apply     # read at construction (fast_gp_digital_net_b2.py:226)
        alt = run(fg, qmcpy, family)
        qmcpy.fftbr_torch, qmcpy.ifftbr_torch, qmcpy.fwht_torch = keep
        lh_r, lh_a = ref["loss_hist"], alt["loss_hist"]
        spread[name] = {
            "config": "%s n=2^%d d=%d alpha=2, default nugget, fit(iterations=%d, stop_crit_wait_iterations=%d), "
                      "post_mean N=%d, post_var N=%d" % ("C2 FastGPLattice" if family == "lattice" else
                                                         "C3 FastGPDigitalNetB2", M, D, ITS, ITS + 1, NM, NV),
            "what": "the REAL reference (tests/golden/make_golden_c23.py) with " +
                    ("qmcpy.fftbr_torch/ifftbr_torch (torch.fft) vs numpy pocketfft" if family == "lattice" else
                     "the stand-in's fwht_torch vs a reverse-stage-order butterfly with per-stage 1/sqrt(2)"),
            "loss_hist_rel": rel(lh_a, lh_r),
            "loss_hist_rel_per_iteration_max": float(np.max(np.abs(lh_a - lh_r) / np.abs(lh_r))),
            "raw_lengthscales_abs": float(np.max(np.abs(alt["raw_lengthscales"] - ref["raw_lengthscales"]))),
            "raw_scale_abs": float(np.max(np.abs(alt["raw_scale"] - ref["raw_scale"]))),
            "pmean_rel": rel(alt["pmean"], ref["pmean"]),
            "pvar_abs_over_kxx": float(np.max(np.abs(alt["pvar"] - ref["pvar"]) / np.abs(ref["kxx"])))}
    with open(os.path.join(ROOT, "profiles", "r06_c23_backend_spread.json"), "w") as f:
        json.dump(spread, f, indent=1)
    print(json.dumps(spread, indent=1))


if __name__ == "__main__":
    main()
