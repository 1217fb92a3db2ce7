"""Batches of independent fast GPs (e.g. the randomly shifted replicas of one lattice GP, BASELINE
config C4) fitted and predicted in ONE device-resident launch sequence.

fastgps fits and predicts each GP on its own (AbstractGP.fit / post_mean / post_var,
fastgps/abstract_gp.py:152-416).  On MI355X a single n = 2^20 GP fills only 256 workgroups per
transform pass, and a per-GP predict is a chain of small launches, so independent GPs of the same
family / n / d / smoothness are stacked: one fgp_fit_run with P problems (per_problem mode: every GP
keeps its own loss, Rprop state and early-stopping decision), one batched coefficient solve, one
posterior-mean and one posterior-variance launch for all P GPs.  The result for each GP is what its
own methods return: the stopping rule is applied per GP on its own loss history, each GP's best
parameters are restored, and the GP objects hold the fitted parameters and data afterwards.
"""
import collections
import ctypes
import math

import torch

from . import _native as N
from . import ops
from .fit_engine import FusedMLL, LatticePartsGen, cached_engine, fused_lam, mll_constant, spec_basis, spec_basis_gen, spec_inv_eig, spectral_wanted


class _LossReader(object):
    """Pipelined read-back of the loss history: each enqueued chunk of fit iterations is copied to
    pinned host memory on a side stream once an event recorded after it fires, so reading chunk k
    never waits for the chunks enqueued after it (the device loop keeps running)."""

    def __init__(self, device):
        self.side = torch.cuda.Stream(device)

    def submit(self, src):
        ev = torch.cuda.Event()
        ev.record()
        host = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            host.copy_(src, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.side)
        return host, done

    @staticmethod
    def get(item):
        host, done = item
        done.synchronize()
        return host


def _fit_loop(eng, iterations, stop_crit_improvement_threshold, stop_crit_wait_iterations):
    """AbstractGP.fit's iteration / early-stopping rule (fastgps/abstract_gp.py:241-289) applied per
    problem of a per_problem FusedMLL.  Chunks of iterations are enqueued ahead while no problem can
    have stopped before them (a problem that has waited w iterations stops at the earliest after
    wait - w more), so the host reads losses without draining the device queue; iterations a problem
    runs after its stop are discarded (its parameters are restored from the history)."""
    logtol = math.log(1 + stop_crit_improvement_threshold)
    wait_max = stop_crit_wait_iterations
    P = eng.G
    total = iterations + 1
    eng.ensure_history(total)
    if wait_max > iterations:
        # no problem can stop early: every one runs to `iterations` and restores its best iterate
        # (the first minimum of its loss history).  Nothing to decide on the host -> no host sync; the
        # best iterations are found on the device (_best_raw) and losses are copied back only on request.
        eng.run(0, total, final_no_update=True)
        return [dict(stop=iterations, best_i=None, losses=None, p=p, eng=eng) for p in range(P)]
    reader = _LossReader(eng.device)
    state = [dict(best=math.inf, save=math.inf, waited=0, best_i=0, stop=None, losses=[]) for _ in range(P)]
    pending = collections.deque()
    enq = read = 0
    chunk = 4
    while True:
        active = [s for s in state if s["stop"] is None]
        if not active:
            break
        while enq < total and (enq == read or all(wait_max - s["waited"] > enq - read for s in active)):
            k = min(chunk, total - enq)
            eng.run(enq, k, final_no_update=(enq + k == total))
            pending.append((enq, k, reader.submit(eng.loss_hist[enq:enq + k])))
            enq += k
            chunk = min(64, chunk * 2)
        i0, k, item = pending.popleft()
        lh = _LossReader.get(item)
        for p, s in enumerate(state):
            if s["stop"] is not None:
                continue
            for r in range(k):
                i = i0 + r
                lv = float(lh[r, p, 0])
                s["losses"].append(lv)
                if lv < s["best"]:
                    s["best"], s["best_i"] = lv, i
                if (s["save"] - lv) > logtol:
                    s["waited"] = 0
                    s["save"] = s["best"]
                else:
                    s["waited"] += 1
                if i == iterations or s["waited"] == wait_max:
                    s["stop"] = i
                    break
        read = i0 + k
    for _, _, item in pending:          # drain speculative chunks' copies
        _LossReader.get(item)
    return state


_COLS = {}


def _best_cols(device, P, S, L, dl):
    """The raw-vector columns of every problem's (scale, lengthscales, noise), a device tensor made once per
    shape (no host-to-device copy in a step: a hipGraph capture of the step cannot take one)."""
    key = (str(device), P, S, L, dl)
    if key not in _COLS:
        cols = []
        for p in range(P):
            cols += [p] + [S + p * dl + j for j in range(dl)] + [S + L + p]
        _COLS[key] = torch.tensor(cols, dtype=torch.int64).to(device)
    return _COLS[key]


def _best_raw(eng, state, dl):
    """[P, 2 + dl] = (raw scale, raw lengthscales, raw noise) of every problem at its best iteration
    (one gather from the per-iteration parameter history).  Best iterations decided on the device
    (best_i None: the first minimum of each loss history, = the host rule `lv < best`) stay there."""
    P = eng.G
    S, L, _ = eng.sizes
    idx_c = _best_cols(eng.device, P, S, L, dl)
    if state[0]["best_i"] is None:
        total = state[0]["stop"] + 1
        lh = eng.loss_hist[:total, :, 0]
        lh = torch.where(torch.isnan(lh), torch.full_like(lh, math.inf), lh)   # NaN never becomes best
        best = lh.argmin(0)                                                 # [P], first minimum
        idx_r = best.repeat_interleave(2 + dl)
    else:
        rows = []
        for s in state:
            rows += [s["best_i"]] * (2 + dl)
        idx_r = torch.tensor(rows, dtype=torch.int64).pin_memory().to(eng.device, non_blocking=True)
    return eng.raw_hist[idx_r, idx_c].reshape(P, 2 + dl)


def _check_batch(gps):
    assert len(gps) > 0
    g0 = gps[0]
    n = g0._nh
    for gp in gps:
        assert type(gp) is type(g0), "a GP batch needs GPs of one family"
        assert gp._nh == n and gp.d == g0.d and gp._alphas == g0._alphas and gp.device == g0.device
        assert gp._fused_ok(), "every GP must qualify for the fused MLL path"
        assert gp._problem_batch()[1] == 1, "per-output hyper-parameters: fit those GPs individually"
        assert gp.raw_lengthscales.shape == g0.raw_lengthscales.shape
        assert (gp.raw_scale.requires_grad, gp.raw_lengthscales.requires_grad, gp.raw_noise.requires_grad) == \
               (g0.raw_scale.requires_grad, g0.raw_lengthscales.requires_grad, g0.raw_noise.requires_grad)
    return g0, n


def _parts_source(gps, n):
    """Lattice GPs sharing one generating vector regenerate their parts in the kernels (only the P
    shifts are stacked); otherwise a stacked [P, d, n] parts array."""
    gens = [gp._parts_gen(n) for gp in gps]
    if all(g is not None for g in gens) and all(g.z == gens[0].z for g in gens):
        return None, LatticePartsGen(gens[0].z, gens[0].alphas, torch.cat([g.shift for g in gens], 0))
    g0 = gps[0]
    parts = torch.empty((len(gps), g0.d, n), dtype=torch.float64, device=g0.device)
    for p, gp in enumerate(gps):
        gp._k1parts(n, out=parts[p])
    return parts, None


def _set_raw(gps, raw, dl):
    """Install raw[p] = (scale, lengthscales, noise) as GP p's raw parameters (views: no copies)."""
    for p, gp in enumerate(gps):
        vals = {"raw_scale": raw[p, 0:1], "raw_lengthscales": raw[p, 1:1 + dl], "raw_noise": raw[p, 1 + dl:2 + dl]}
        for name, v in vals.items():
            old = getattr(gp, name)
            setattr(gp, name, torch.nn.Parameter(v.reshape(old.shape), requires_grad=old.requires_grad))
        gp._cache = {k: v for k, v in gp._cache.items() if not k[2]}
        gp._snap = None


def _basis_for(gps, n, parts, gen):
    """Part-product spectra of the batch (fit_engine.spec_basis) when the spectral fit path is the cheaper
    one, else None: ONE set for lattice GPs sharing a generating vector (the first-column
    distances (brev(i) z mod n) / n do not depend on the shift), else [P, 2^d, K] from the stacked parts."""
    g0 = gps[0]
    P = len(gps)
    shared = gen is not None or P == 1
    if not spectral_wanted(g0._FAMILY, n, g0.d, P, 1 if shared else P):
        return None
    if gen is not None:
        b = spec_basis_gen(gen, n, g0.device)                  # the parts regenerated in the transform
        if b is not None:
            return b
        p = ops.lattice_parts_gen(gen.z, gen.shift[0], gen.alphas, n)
    else:
        p = parts[0] if P == 1 else parts
    return spec_basis(g0._FAMILY, p, n)


def _engine(gps, n, ysq, parts, gen, lr, iterations, basis=None, cached=False):
    g0 = gps[0]
    dl = g0.raw_lengthscales.shape[-1]
    d_out = int(math.prod(g0.shape_batch))
    if cached and basis is not None:
        # the batch's spectral engine, reused across fits of this geometry (fit_engine.cached_engine)
        return cached_engine(g0._FAMILY, ysq, torch.stack([gp.raw_scale.detach().reshape(-1)[0] for gp in gps]),
                             torch.stack([gp.raw_lengthscales.detach().reshape(dl) for gp in gps]),
                             torch.stack([gp.raw_noise.detach().reshape(-1)[0] for gp in gps]),
                             logdet_weight=float(d_out), mll_const=mll_constant(d_out, n),
                             requires_grad=(g0.raw_scale.requires_grad, g0.raw_lengthscales.requires_grad,
                                            g0.raw_noise.requires_grad),
                             lr=1e-1 if lr is None else lr, max_iters=iterations + 1, basis=basis, per_problem=True)
    return FusedMLL(g0._FAMILY, parts, ysq,
                    torch.stack([gp.raw_scale.detach().reshape(-1)[0] for gp in gps]),
                    torch.stack([gp.raw_lengthscales.detach().reshape(dl) for gp in gps]),
                    torch.stack([gp.raw_noise.detach().reshape(-1)[0] for gp in gps]),
                    logdet_weight=float(d_out), mll_const=mll_constant(d_out, n),
                    requires_grad=(g0.raw_scale.requires_grad, g0.raw_lengthscales.requires_grad,
                                   g0.raw_noise.requires_grad),
                    lr=1e-1 if lr is None else lr, max_iters=iterations + 1, parts_per_problem=True,
                    per_problem=True, gen=None if basis is not None else gen,
                    basis=basis)


def _fit_data(state, store):
    out = []
    lh = None
    for s in state:
        data = {"iterations": s["stop"]}
        if store:
            if s["losses"] is None:          # device-decided run: copy the histories back now
                if lh is None:
                    lh = s["eng"].loss_hist[:s["stop"] + 1, :, 0].cpu()
                data["loss_hist"] = -lh[:, s["p"]].clone()
            else:
                data["loss_hist"] = torch.tensor([-v for v in s["losses"]])
        out.append(data)
    return out


def fit_batched(gps, iterations=5000, lr=None, stop_crit_improvement_threshold=5e-2, stop_crit_wait_iterations=10,
                store_hists=False, store_loss_hist=False):
    """Fit independent single-problem GPs (same class, n, d, alpha, shapes) with the fused MLL loop.

    Returns the list of per-GP `data` dicts that `gp.fit(iterations=..., verbose=0, ...)` would return."""
    g0, n = _check_batch(gps)
    eng = batched_engine(gps, iterations, lr)
    state = _fit_loop(eng, iterations, stop_crit_improvement_threshold, stop_crit_wait_iterations)
    _set_raw(gps, _best_raw(eng, state, g0.raw_lengthscales.shape[-1]).clone(), g0.raw_lengthscales.shape[-1])
    return _fit_data(state, store_hists or store_loss_hist)


def batched_engine(gps, iterations, lr=None):
    """The FusedMLL (per_problem mode) over the GPs' stacked problems: Y = |ytilde|^2 rows and raw
    parameters stacked, the kernel parts regenerated in the kernels for lattice GPs sharing one
    generating vector (otherwise a stacked [P, d, n] parts array)."""
    n = gps[0]._nh
    parts, gen = _parts_source(gps, n)
    ysq = torch.stack([gp._ysq(*gp._problem_batch())[0] for gp in gps])
    return _engine(gps, n, ysq, parts, gen, lr, iterations, basis=_basis_for(gps, n, parts, gen))


class GPBatch(object):
    """P independent single-output fast GPs of one family, n, d and smoothness held in stacked device
    buffers: ytilde [P, n], Y = |ytilde|^2, training points [P, d, n] (each GP's cached dimension-major
    points become views of it), fitted raw parameters [P, 2 + dl], coefficients [P, n] and the
    eigenvalue weights Re(1/ev) [P, n].  Methods mirror the per-GP API and return [P, ...] stacks."""

    def __init__(self, gps):
        gps = list(gps)
        g0, n = _check_batch(gps)
        for gp in gps:
            assert gp.shape_batch == torch.Size([]), "GPBatch holds single-output GPs"
        self.gps = gps
        self.P = len(gps)
        self.n = n
        self.m = ops.log2_exact(n)
        self.d = g0.d
        self.family = g0._FAMILY
        self.device = g0.device
        self.dl = g0.raw_lengthscales.shape[-1]
        self.z = torch.empty((self.P, self.d, n), dtype=g0._XBDTYPE, device=self.device)
        for p, gp in enumerate(gps):
            self.z[p].copy_(gp._points_T(n))
            gp._pts_T = (n, self.z[p])
        self.part0 = [float(v) for v in g0._part_at_zero()]
        self.tbits = g0._tbits()
        self._n_t = torch.tensor([n], dtype=torch.int64, device=self.device)
        self._m_t = torch.tensor([self.m], dtype=torch.int64, device=self.device)
        self._y = None
        self._st = {}
        self._src = None
        self._unit_ok = {}

    # ---------------------------------------------------------------------------- data / parameters
    def set_data(self, y):
        """Give GP p the observations y[p] at its n points ([P, n]): AbstractGP.add_y_next
        (fastgps/abstract_gp.py:331-351) on GPs without data, for all P at once."""
        y = y.to(device=self.device, dtype=torch.float64)
        assert y.shape == (self.P, self.n)
        for p, gp in enumerate(self.gps):
            gp._y[0] = y[p]
            gp._nh = self.n
            gp.n, gp.m = self._n_t, self._m_t
            gp._cache = {}
            gp._yt_state = None
        self._y = y
        self._st = {}

    def set_raw(self, raw):
        """Set every GP's raw (log) hyper-parameters from raw [P, 2 + dl] = (scale, lengthscales, noise)."""
        assert raw.shape == (self.P, 2 + self.dl)
        _set_raw(self.gps, raw, self.dl)
        for k in ("raw", "coeffs", "wa", "hyp"):
            self._st.pop(k, None)
        self._put_ytilde()

    def raw(self):
        if "raw" not in self._st:
            self._st["raw"] = torch.stack([torch.cat([gp.raw_scale.detach().reshape(1),
                                                      gp.raw_lengthscales.detach().reshape(self.dl),
                                                      gp.raw_noise.detach().reshape(1)]) for gp in self.gps])
        return self._st["raw"]

    def _source(self):
        if self._src is None:
            self._src = _parts_source(self.gps, self.n)
        return self._src

    def basis(self):
        """The batch's part-product spectra (None: transform fit path); rebuilt after set_data, like every
        other cache of a step."""
        if "basis" not in self._st:
            parts, gen = self._source()
            self._st["basis"] = _basis_for(self.gps, self.n, parts, gen)
        return self._st["basis"]

    def _put_ytilde(self):
        yt, yth = self._st.get("yt"), self._st.get("yth")
        for p, gp in enumerate(self.gps):
            if yt is not None:
                gp._cache[("ytilde", self.n, False, False)] = yt[p]
            if yth is not None:
                gp._cache[("ytilde_half", self.n, False, False)] = yth[p]

    def _y_rows(self):
        return self._y if self._y is not None else torch.stack([gp._y[0] for gp in self.gps])

    def ytilde_half(self):
        """[P, n/2 + 1] Hermitian halves of ytilde (lattice, real fp64 observations, 2^17 <= n <= 2^24;
        ops.fftbr_real_half): all that Y and the spectral coefficient solve read.  None when it does not apply."""
        if "yth" not in self._st:
            if "yt" in self._st:
                return self._st["yt"][:, :self.n // 2 + 1] if self.family == ops.LATTICE else None
            y = self._y_rows()
            if self.family != ops.LATTICE or not ops.half_spectrum_ok(y):
                return None
            self._st["yth"] = ops.fftbr_real_half(y)
            self._put_ytilde()
        return self._st["yth"]

    def ytilde(self):
        """[P, n] ytilde = ft(y) of every GP (AbstractFastGP.get_ytilde / _YtildeCache, util.py:164-183),
        one batched transform (or the mirror of the Hermitian halves when only those were formed); also
        installed in each GP's cache."""
        if "yt" not in self._st:
            if "yth" in self._st:
                yt = ops.hermitian_full(self._st["yth"], self.n)
            elif self.family == ops.LATTICE:
                yt = ops.fftbr_raw(self._y_rows(), stable=True)
            else:
                yt = ops.fwht_raw(self._y_rows(), stable=True)
            self._st["yt"] = yt
            self._put_ytilde()
        return self._st["yt"]

    def ysq(self):
        if "ysq" not in self._st:
            yth = self.ytilde_half()
            if yth is not None:                                 # |ytilde|^2 per GP from the halves (fgp_sum_sq_half)
                self._st["ysq"] = ops.sum_sq_half(yth, self.n, G=self.P)
            else:
                self._st["ysq"] = ops.sum_sq(self.ytilde(), G=self.P)   # (fgp_sum_sq)
        return self._st["ysq"]

    # ---------------------------------------------------------------------------- fit
    def fit(self, iterations=5000, lr=None, stop_crit_improvement_threshold=5e-2, stop_crit_wait_iterations=10,
            store_hists=False, store_loss_hist=False):
        """Every GP's AbstractGP.fit(loss_metric="MLL", verbose=0) in one device loop; returns the list of
        per-GP data dicts."""
        parts, gen = self._source()
        eng = _engine(self.gps, self.n, self.ysq(), parts, gen, lr, iterations, basis=self.basis(), cached=True)
        state = _fit_loop(eng, iterations, stop_crit_improvement_threshold, stop_crit_wait_iterations)
        best = _best_raw(eng, state, self.dl)
        self.set_raw(best)
        self._st["raw"] = best
        out = _fit_data(state, store_hists or store_loss_hist)
        eng.release_inputs()
        return out

    # ---------------------------------------------------------------------------- predict
    def coeffs(self):
        """[P, n] K^-1 y of every GP (_CoeffsCache, util.py:396-425): lambda by fgp_nll_lam, A = 1/ev and
        ytilde * A by fgp_inv_eig, one batched inverse transform."""
        if "coeffs" not in self._st:
            raw = self.raw()
            parts, gen = self._source()
            dl = self.dl
            basis = self.basis()
            if basis is not None and self.family == ops.LATTICE and 17 <= self.m <= 24:
                # spectral path: A = 1/ev straight from the spectra (real), the product fused into the
                # half-length inverse -- no lambda / ytilde * A arrays
                wa = spec_inv_eig(self.family, raw[:, 0], raw[:, 1:1 + dl], raw[:, 1 + dl], self.P, self.n, basis)
                yth = self.ytilde_half()
                self._st["coeffs"] = ops.ifftbr_real_rf(yth if yth is not None else self.ytilde(), wa, n=self.n)
                self._st["wa"] = wa
                return self._st["coeffs"]
            lam = fused_lam(self.family, parts, raw[:, 0], raw[:, 1:1 + dl], raw[:, 1 + dl], self.P, gen=gen, n=self.n,
                            basis=self.basis())
            yt = self.ytilde()
            ya = torch.empty_like(lam)
            wa = torch.empty((self.P, self.n), dtype=torch.float64, device=self.device)
            noise = raw[:, 1 + dl:]
            N.call("fgp_inv_eig", self.family, N.ptr(lam), N.ptr(yt), yt.stride(0), N.ptr(noise), raw.stride(0),
                   self.P, self.m, N.ptr(ya), N.ptr(wa), N.stream_ptr(self.device))
            if self.family == ops.LATTICE:
                self._st["coeffs"] = ops.ifftbr_raw(ya, stable=True, real_out=True)
            else:
                self._st["coeffs"] = ops.fwht_raw(ya, stable=True)
            self._st["wa"] = wa
        return self._st["coeffs"]

    def _hyp(self):
        if "hyp" not in self._st:
            h = torch.exp(self.raw()[:, :1 + self.dl])
            if self.dl != self.d:
                h = torch.cat([h[:, :1], h[:, 1:2].expand(self.P, self.d)], 1)
            self._st["hyp"] = h.contiguous()
        return self._st["hyp"]

    def _desc(self):
        order, coef = ops._pred_args(self.family, self.gps[0]._alphas, self.d)
        hyp = self._hyp()
        coeffs = self._st["coeffs"]
        wa = self._st["wa"]
        desc = N.PredDesc(family=self.family, d=self.d, tbits=int(self.tbits), P=self.P, n=self.n,
                          z=self.z.data_ptr(), z_stride=self.d * self.n, hyp=hyp.data_ptr(), hyp_stride=hyp.stride(0),
                          coeffs=coeffs.data_ptr(), coeff_stride=coeffs.stride(0), wa=wa.data_ptr(),
                          wa_stride=wa.stride(0))
        for j in range(self.d):
            desc.order[j] = order[j]
            desc.coef[j] = coef[j]
        _, gen = self._source()
        if gen is not None:     # post_var regenerates the lattice points instead of reading z
            desc.points_gen = N.PARTS_LATTICE
            for j in range(self.d):
                desc.gen_z[j] = gen.z[j]
            desc.gen_shift = gen.shift.data_ptr()
            desc.gen_shift_stride = self.d if gen.shift.shape[0] > 1 else 0
        return desc

    def _points(self, x):
        x = x.to(device=self.device, dtype=torch.float64)
        assert (x.ndim == 2 and x.size(1) == self.d) or (x.ndim == 3 and x.shape[0] == self.P and x.size(2) == self.d), \
            "x must have shape (N, d) (shared) or (P, N, d)"
        x = x.contiguous()
        # the [0, 1] range check of the reference (fast_gp_lattice.py:264-265) synchronises; a tensor
        # already checked (same storage, version, shape) is not checked again (the tensor is held)
        key = (x.data_ptr(), x._version, tuple(x.shape))
        if key not in self._unit_ok:
            assert bool(((0 <= x) & (x <= 1)).all()), "x should have all elements in [0,1]"
            self._unit_ok[key] = x
            if len(self._unit_ok) > 8:
                self._unit_ok.pop(next(iter(self._unit_ok)))
        return x, (0 if x.ndim == 2 else x.stride(0)), x.shape[-2]

    def post_mean(self, x):
        """[P, N] posterior means (AbstractGP.post_mean of every GP, abstract_gp.py:352-380)."""
        self.coeffs()
        x, xs, Nt = self._points(x)
        desc = self._desc()
        wl = ctypes.c_int64(0)
        N.call("fgp_post_mean_batched_work", desc, Nt, ctypes.byref(wl))
        work = torch.empty(wl.value, dtype=torch.float64, device=self.device)
        out = torch.empty((self.P, Nt), dtype=torch.float64, device=self.device)
        N.call("fgp_post_mean_batched", desc, N.ptr(x), xs, Nt, N.ptr(out), N.ptr(work),
               N.stream_ptr(self.device))
        return out

    def post_var(self, x, chunk=16):
        """[P, N] posterior variances at the GPs' current n (AbstractGP.post_var, abstract_gp.py:381-416)."""
        if self.m < 13:
            return torch.stack([gp.post_var(x) for gp in self.gps])
        self.coeffs()
        x, xs, Nt = self._points(x)
        out = torch.empty((self.P, Nt), dtype=torch.float64, device=self.device)
        cdt = torch.complex128 if self.family == ops.LATTICE else torch.float64
        desc = self._desc()
        part0 = N.double_array(self.part0)
        for t0 in range(0, Nt, chunk):
            t1 = min(Nt, t0 + chunk)
            xc = x[..., t0:t1, :].contiguous()
            work = torch.empty((self.P, t1 - t0, self.n), dtype=cdt, device=self.device)
            partial = torch.empty((self.P, t1 - t0, self.n >> 12), dtype=torch.float64, device=self.device)
            oc = torch.empty((self.P, t1 - t0), dtype=torch.float64, device=self.device)
            N.call("fgp_post_var_batched", desc, N.ptr(xc), (0 if xc.ndim == 2 else xc.stride(0)), t1 - t0, part0,
                   N.ptr(oc), N.ptr(work), N.ptr(partial), N.stream_ptr(self.device))
            out[:, t0:t1] = oc
        return out
