"""Golden vectors for the BENCHED C5 regime (BASELINE config C5: multi-output FastGPLattice, n = 2^18,
d = 3, 512 outputs, shared hyper-parameters, the default nugget 1e-8), from the REAL reference, and the
reference's own FFT-backend sensitivity there (VERDICT r02 "Next round" item 1).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c5.py

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c5.py --per-output

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c5.py [--per-output] --its 50

--its 50 (round 6): the benched length, fit(iterations=50, stop_crit_wait_iterations=51), written to the *_it50.npz
fixtures and profiles/r06_c5*_backend_spread.json.

Writes tests/golden/c5_m18_d3_b512.npz (inputs: the point set's generating vector + shift and the data
seed; outputs: the reference's fit(iterations=3) loss / parameter trajectory, post_mean at 16 test points,
post_var at 2), tests/golden/c5_m18_d3_b512_f32data.npz (the same on the observations rounded to float32:
the mixed-precision path's data) and profiles/r03_c5_backend_spread.json: the same run with the reference's qmcpy
fftbr_torch / ifftbr_torch replaced by numpy's pocketfft (a differentiable wrapper, adjoints by the
inverse transform) -- the spread a correct implementation of the reference can show at this size and
nugget.  tests/test_gpu_multioutput.py allows 5x it.

--per-output: the benched per-output regime instead (docs/examples/batch_multitask/fgp_lattice.ipynb
cell 6: shape_scale = [512, 1], shape_lengthscales = [512, 3] -- 512 independent eigen-problems on one point
set, one summed loss; nugget 1e-8): tests/golden/c5_m18_d3_b512_po.npz and
profiles/r04_c5_po_backend_spread.json.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from oracle.refshim.load_reference import import_reference  # noqa: E402
from make_golden import LATTICE_Z, f_ackley  # noqa: E402

M, D, B, NM, NV = 18, 3, 512, 16, 2
# --its N: the fit length (3: the original fixtures; 50: the benched length, VERDICT r05 item 1 -- files and spread
# records then carry the suffix _it50 / r06_)
ITS = int(sys.argv[sys.argv.index("--its") + 1]) if "--its" in sys.argv else 3
SUF = "" if ITS == 3 else "_it%d" % ITS
STOP = ITS + 5 if ITS == 3 else ITS + 1      # early stopping off either way


def c5_data(x, B, seed=5):
    """y_b = f_ackley(x) (1 + b / B) + 0.01 randn (CPU generator, seeded): bench.py's C5 shape."""
    f = f_ackley(x)
    g = torch.Generator().manual_seed(seed)
    noise = torch.randn((B, x.shape[0]), generator=g, dtype=torch.float64)
    b = torch.arange(B, dtype=torch.float64)[:, None]
    return f[None, :] * (1 + b / B) + 0.01 * noise


def _bitrev(n):
    m = n.bit_length() - 1
    i = np.arange(n)
    r = np.zeros(n, dtype=np.int64)
    for k in range(m):
        r |= ((i >> k) & 1) << (m - 1 - k)
    return torch.from_numpy(r)


class _NpFFTBR(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        br = _bitrev(x.size(-1))
        ctx.real = not x.is_complex()
        return torch.from_numpy(np.fft.fft(x[..., br].detach().numpy(), norm="ortho"))

    @staticmethod
    def backward(ctx, g):
        br = _bitrev(g.size(-1))
        gx = torch.from_numpy(np.fft.ifft(g.detach().numpy(), norm="ortho"))[..., br]
        return gx.real if ctx.real else gx


class _NpIFFTBR(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        br = _bitrev(x.size(-1))
        ctx.real = not x.is_complex()
        return torch.from_numpy(np.fft.ifft(x.detach().numpy(), norm="ortho"))[..., br]

    @staticmethod
    def backward(ctx, g):
        br = _bitrev(g.size(-1))
        gx = torch.from_numpy(np.fft.fft(g[..., br].detach().numpy(), norm="ortho"))
        return gx.real if ctx.real else gx


def run(fg, qmcpy, backend, f32_data=False):
    if backend == "numpy":
        qmcpy.fftbr_torch, qmcpy.ifftbr_torch = _NpFFTBR.apply, _NpIFFTBR.apply
    n = 2 ** M
    shift = np.random.default_rng(7).uniform(size=D)
    seq = qmcpy.Lattice(D, randomize="SHIFT", generating_vector=LATTICE_Z[:D], shift=shift)
    gp = fg.FastGPLattice(seq, alpha=2, shape_batch=[B])
    x = gp.get_x_next(n)
    y = c5_data(x, B)
    if f32_data:     # the mixed-precision C5 path's observations (data_dtype=float32), fp64 from there on
        y = y.float().double()
    gp.add_y_next(y)
    data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=STOP)
    xt = torch.rand((NM, D), generator=torch.Generator().manual_seed(17))
    pm = gp.post_mean(xt)
    pv = gp.post_var(xt[:NV])
    return dict(z=np.array(LATTICE_Z[:D], dtype=np.int64), shift=shift, x_test=xt.numpy(),
                loss_hist=data["loss_hist"].detach().numpy(),
                raw_scale=gp.raw_scale.detach().numpy(), raw_lengthscales=gp.raw_lengthscales.detach().numpy(),
                pmean=pm.detach().numpy(), pvar=pv.detach().numpy(),
                kxx=float(gp.kernel(xt[:NV], xt[:NV]).detach().abs().max()))


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / np.max(np.abs(np.asarray(b))))


PO_CHUNK = 64


def run_per_output(fg, qmcpy, backend):
    """The per-output regime through the REAL reference, in chunks of PO_CHUNK outputs: the reference's
    per-output problems are independent (Rprop steps every parameter element on its own gradient, the loss
    is the sum of the per-output MLLs with logdet weight d_out / numel(logdet) = 1 and constant d_out n
    log 2 pi), so the 512-output run is the concatenation of the chunks' parameters / posteriors and the sum
    of their loss histories -- at 1/8 of the reference's memory (one 512-output autograd graph does not fit
    this container's 64 GB).  Each chunk gets its rows of the full [512, n] observations."""
    if backend == "numpy":
        qmcpy.fftbr_torch, qmcpy.ifftbr_torch = _NpFFTBR.apply, _NpIFFTBR.apply
    n = 2 ** M
    shift = np.random.default_rng(7).uniform(size=D)
    outs = []
    yfull = None
    for a in range(0, B, PO_CHUNK):
        Bc = min(PO_CHUNK, B - a)
        seq = qmcpy.Lattice(D, randomize="SHIFT", generating_vector=LATTICE_Z[:D], shift=shift)
        gp = fg.FastGPLattice(seq, alpha=2, shape_batch=[Bc], shape_scale=[Bc, 1], shape_lengthscales=[Bc, D])
        x = gp.get_x_next(n)
        if yfull is None:
            yfull = c5_data(x, B)
        gp.add_y_next(yfull[a:a + Bc].clone())
        data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=STOP)
        xt = torch.rand((NM, D), generator=torch.Generator().manual_seed(17))
        pm = gp.post_mean(xt)
        pv = gp.post_var(xt[:NV])
        outs.append(dict(loss_hist=data["loss_hist"].detach().numpy(), raw_scale=gp.raw_scale.detach().numpy(),
                         raw_lengthscales=gp.raw_lengthscales.detach().numpy(), pmean=pm.detach().numpy(),
                         pvar=pv.detach().numpy(), kxx_all=gp.kernel(xt[:NV], xt[:NV]).detach().numpy(),
                         x_test=xt.numpy()))
        del gp, data
        print("chunk", a, "done", flush=True)
    cat = lambda k: np.concatenate([o[k] for o in outs], 0)
    return dict(z=np.array(LATTICE_Z[:D], dtype=np.int64), shift=shift, x_test=outs[0]["x_test"],
                loss_hist=np.sum([o["loss_hist"] for o in outs], 0), raw_scale=cat("raw_scale"),
                raw_lengthscales=cat("raw_lengthscales"), pmean=cat("pmean"), pvar=cat("pvar"),
                kxx_all=cat("kxx_all"), chunk=np.array(PO_CHUNK))


def main_per_output(fg, qmcpy):
    keep = (qmcpy.fftbr_torch, qmcpy.ifftbr_torch)
    path = os.path.join(HERE, "c5_m18_d3_b512_po%s.npz" % SUF)
    if "--reuse" in sys.argv and os.path.isfile(path):      # the torch-backend fixture of an earlier run
        ref = dict(np.load(path))
    else:
        ref = run_per_output(fg, qmcpy, "torch")
        np.savez_compressed(path, m=np.array(M), d=np.array(D), B=np.array(B), its=np.array(ITS),
                            **{k: np.asarray(v) for k, v in ref.items()})
    alt = run_per_output(fg, qmcpy, "numpy")
    qmcpy.fftbr_torch, qmcpy.ifftbr_torch = keep
    if ITS != 3:
        # over 50 iterations the sign-driven Rprop trajectories of some outputs fork between the two backends: the
        # pocketfft run's per-output results are kept too (tests/test_gpu_multioutput.py pins each output to the
        # reference run it follows)
        np.savez_compressed(os.path.join(HERE, "c5_m18_d3_b512_po%s_alt.npz" % SUF),
                            **{k: np.asarray(alt[k]) for k in ("loss_hist", "raw_scale", "raw_lengthscales", "pmean",
                                                                "pvar")})
    kdiag = np.abs(ref["kxx_all"])        # [B, NV]: each output's own K(x_t, x_t) (per-output scales)
    spread = {"config": "C5 per-output: lattice n=2^%d d=%d x %d outputs, shape_scale=[%d,1], "
                        "shape_lengthscales=[%d,%d], nugget 1e-8, fit(iterations=%d), post_mean N=%d, post_var N=%d"
                        % (M, D, B, B, B, D, ITS, NM, NV),
              "what": "the REAL reference (tests/golden/make_golden_c5.py --per-output, chunks of %d outputs) with "
                      "qmcpy.fftbr_torch/ifftbr_torch (torch.fft) vs numpy pocketfft" % PO_CHUNK,
              "loss_hist_rel": rel(alt["loss_hist"], ref["loss_hist"]),
              "raw_lengthscales_abs": float(np.max(np.abs(alt["raw_lengthscales"] - ref["raw_lengthscales"]))),
              "raw_scale_abs": float(np.max(np.abs(alt["raw_scale"] - ref["raw_scale"]))),
              "pmean_rel": rel(alt["pmean"], ref["pmean"]),
              "pvar_abs_over_kxx": float(np.max(np.abs(alt["pvar"] - ref["pvar"]) / kdiag))}
    same = np.all(np.abs(alt["raw_lengthscales"] - ref["raw_lengthscales"]).reshape(B, -1) == 0, 1) & \
        np.all(np.abs(alt["raw_scale"] - ref["raw_scale"]).reshape(B, -1) == 0, 1)
    spread["outputs_same_parameters"] = int(same.sum())
    spread["outputs_forked"] = [int(b) for b in np.nonzero(~same)[0]]
    if same.any():
        spread["pmean_rel_unforked"] = rel(alt["pmean"][same], ref["pmean"][same])
        spread["pvar_abs_over_kxx_unforked"] = float(np.max(np.abs(alt["pvar"][same] - ref["pvar"][same]) / kdiag[same]))
    with open(os.path.join(ROOT, "profiles", "r04_c5_po_backend_spread.json" if ITS == 3 else "r06_c5_po_backend_spread.json"), "w") as f:
        json.dump(spread, f, indent=1)
    print(json.dumps(spread, indent=1))


def main():
    torch.set_default_dtype(torch.float64)
    torch.set_num_threads(os.cpu_count() or 1)
    fg = import_reference()
    import qmcpy
    if "--per-output" in sys.argv:
        return main_per_output(fg, qmcpy)
    keep = (qmcpy.fftbr_torch, qmcpy.ifftbr_torch)
    ref = run(fg, qmcpy, "torch")
    np.savez_compressed(os.path.join(HERE, "c5_m18_d3_b512%s.npz" % SUF), m=np.array(M), d=np.array(D), B=np.array(B),
                        its=np.array(ITS), **{k: np.asarray(v) for k, v in ref.items()})
    r32 = run(fg, qmcpy, "torch", f32_data=True)
    np.savez_compressed(os.path.join(HERE, "c5_m18_d3_b512_f32data%s.npz" % SUF), m=np.array(M), d=np.array(D),
                        B=np.array(B), its=np.array(ITS), **{k: np.asarray(v) for k, v in r32.items()})
    alt = run(fg, qmcpy, "numpy")
    qmcpy.fftbr_torch, qmcpy.ifftbr_torch = keep
    spread = {"config": "C5 lattice n=2^%d d=%d x %d outputs, nugget 1e-8, fit(iterations=%d), post_mean N=%d, "
                        "post_var N=%d" % (M, D, B, ITS, NM, NV),
              "what": "the REAL reference (tests/golden/make_golden_c5.py) with qmcpy.fftbr_torch/ifftbr_torch "
                      "(torch.fft) vs numpy pocketfft",
              "loss_hist_rel": rel(alt["loss_hist"], ref["loss_hist"]),
              "raw_lengthscales_abs": float(np.max(np.abs(alt["raw_lengthscales"] - ref["raw_lengthscales"]))),
              "raw_scale_abs": float(np.max(np.abs(alt["raw_scale"] - ref["raw_scale"]))),
              "pmean_rel": rel(alt["pmean"], ref["pmean"]),
              "pvar_abs_over_kxx": float(np.max(np.abs(alt["pvar"] - ref["pvar"])) / ref["kxx"])}
    with open(os.path.join(ROOT, "profiles", "r03_c5_backend_spread.json" if ITS == 3 else "r06_c5_backend_spread.json"), "w") as f:
        json.dump(spread, f, indent=1)
    print(json.dumps(spread, indent=1))


if __name__ == "__main__":
    main()
