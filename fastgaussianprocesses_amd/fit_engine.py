"""Device-resident MLL fit loop (fgp_nll_fwd / fgp_nll_bwd / fgp_fit_step of include/fgp_hip.h).

One `FusedMLL` holds, for G eigen-problems of size n = 2^m:
  * kernel parts [G?, d, n] (shared when parts_stride = 0),
  * Y[g, k] = sum over the outputs of problem g of |ytilde[k]|^2 (the only data the MLL needs),
  * the raw hyper-parameter vector  [raw_scale..., raw_lengthscales..., raw_noise...]  (log scale),
  * workspaces (dL/dlambda, 2-pass intermediate, per-block partials), Rprop state and histories.
`run(iter0, k)` enqueues k complete iterations (forward, adjoint, reduction, Rprop) on the current
stream without any host synchronisation; the caller reads the histories back in chunks to apply
AbstractGP.fit's early-stopping rule (fastgps/abstract_gp.py:276-284) exactly.
"""
import collections
import ctypes
import math
import os

import torch

from . import _native as N
from .ops import LATTICE, lattice_coefficient, log2_exact, require_device

# torch.optim.Rprop defaults (etas=(0.5, 1.2), step_sizes=(1e-6, 50))
RPROP_ETAS = (0.5, 1.2)
RPROP_STEPS = (1e-6, 50.0)


class LatticePartsGen(object):
    """FGP_PARTS_LATTICE parts source (include/fgp_hip.h): the kernels regenerate the lattice parts of
    the natural-order points x_i = ((v(i) z) % 1 + shift) % 1 (seqs.Lattice) instead of reading a
    [d, n] parts array, bit-identically to fgp_lattice_parts on those points.

    z: generating vector [d] (ints); alphas: [d] smoothness; shift: device [S, d] float64 (S = 1 shared
    or one row per problem) holding x[0] (= the shift) of each problem."""

    def __init__(self, z, alphas, shift):
        self.z = [int(v) for v in z]
        self.alphas = [int(a) for a in alphas]
        self.shift = shift.to(torch.float64).reshape(-1, len(self.z)).contiguous()

    def apply(self, desc, n):
        d = len(self.z)
        m = log2_exact(n)
        for j in range(d):
            if not (0 < self.z[j] < 2 ** (53 - m)):
                raise ValueError("generating vector entry outside (0, 2^(53-m))")
        desc.parts_gen = N.PARTS_LATTICE
        for j in range(d):
            desc.gen_order[j] = 2 * self.alphas[j]
            desc.gen_coef[j] = lattice_coefficient(self.alphas[j])
            desc.gen_z[j] = self.z[j]
        desc.gen_shift = self.shift.data_ptr()
        desc.gen_shift_stride = d if self.shift.shape[0] > 1 else 0


FIT_GRAPH_MIN_ITERS = 16       # fgp_fit_run_graph below this many iterations per call: eager launches
_NEXT_TOKEN = 0

SPEC_MAX_D = 6                 # fgp_spec_basis / the spectral fit kernels (include/fgp_hip.h, ABI 11)
SPEC_WORK_CAP = 512 << 20      # scratch of one fgp_spec_basis call (subsets are transformed in chunks)


def spec_k(family, n):
    """Frequencies per part-product spectrum: n/2 + 1 (lattice, real even), n (net)."""
    return n // 2 + 1 if family == 0 else n


def spec_chunks(family, n):
    """64-frequency chunks of the spectra (fgp_spec_basis layout [Q][2^d][64])."""
    return (spec_k(family, n) + 63) // 64


def spec_dense(basis, family, n):
    """[(P,) Q, 2^d, 64] chunked spectra -> [(P,) 2^d, K] (k-contiguous rows; tests / inspection)."""
    t = basis.movedim(-3, -2)
    t = t.reshape(t.shape[:-2] + (t.shape[-2] * 64,))
    return t[..., :spec_k(family, n)]


def spectral_wanted(family, n, d, G, nbases=1):
    """Fit path choice: the part-product spectra (one streaming kernel per iteration, 8 2^d bytes per
    frequency per distinct point set + Y) or the transform kernels (an FFT / FWHT of k1 and its adjoint per
    iteration).  A per-iteration time model from the round-3 measurements:
      spectral:  bytes / 6 TB/s + 6 us;
      transform: max(40 us latency floor of three dependent launches, G n x 10.8 ps (real-even lattice
                 kernels at saturation) / 30 ps (nets, full-length kernels)).
    FGP_FIT_PATH=spectral / transform forces a path (the spectral one needs d <= 6)."""
    if d > SPEC_MAX_D or n < 16:
        return False
    force = os.environ.get("FGP_FIT_PATH", "").lower()
    if force.startswith("s"):
        return True
    if force.startswith("t"):
        return False
    K = spec_k(family, n)
    bytes_it = 8 * K * ((2 ** d) * nbases + G)
    t_spec = bytes_it / 6e12 + 6e-6
    per_point = 10.8e-12 if (family == 0 and n >= 2 ** 16) else 30e-12
    t_tr = max(40e-6, G * n * per_point)
    return t_spec < t_tr and (2 ** d) * nbases * K * 8 <= (16 << 30)


_SPEC_WORK = {}


def _spec_work_bytes(family, m, d):
    """Work bytes of fgp_spec_basis(_gen) for (family, log2 n, d): one subset's transform at least, all 2^d at
    once up to SPEC_WORK_CAP (fgp_spec_basis_work; memoised, a pure function of its arguments)."""
    key = (int(family), int(m), int(d))
    w = _SPEC_WORK.get(key)
    if w is None:
        total = ctypes.c_int64(0)
        N.call("fgp_spec_basis_work", key[0], key[1], key[2], ctypes.byref(total))
        w = _SPEC_WORK[key] = max(total.value >> d, min(total.value, SPEC_WORK_CAP))
    return w


def spec_basis(family, parts, n):
    """Part-product spectra (fgp_spec_basis): parts [d, n] -> [Q, 2^d, 64], or [P, d, n] -> [P, Q, 2^d, 64]
    (chunks of 64 frequencies; spec_dense gives [2^d, K]); lambda = scale sum_S l^S Phi_S for every
    hyper-parameter setting (include/fgp_hip.h)."""
    require_device(parts, "spec_basis")
    parts = parts.contiguous()
    d = parts.shape[-2]
    m = log2_exact(n)
    P = parts.shape[0] if parts.dim() == 3 else 1
    Q = spec_chunks(family, n)
    wbytes = _spec_work_bytes(family, m, d)
    work = torch.empty((wbytes,), dtype=torch.uint8, device=parts.device)
    out = torch.empty(((P,) if parts.dim() == 3 else ()) + (Q, 2 ** d, 64), dtype=torch.float64, device=parts.device)
    N.call("fgp_spec_basis", int(family), N.ptr(parts), d * n, P, m, int(d), N.ptr(out), N.ptr(work), wbytes,
           N.stream_ptr(parts.device))
    return out


def spec_basis_gen(gen, n, device, force=False):
    """spec_basis of lattice parts regenerated from the generating vector inside the transform (fgp_spec_basis_gen,
    ABI 15): the basis of spec_basis(ops.lattice_parts_gen(gen...)) bit for bit, without the d x n parts array;
    None outside its domain (17 <= log2 n <= 24, d <= 6, one smoothness) or with FGP_SPEC_BASIS_GEN=0 (A/B).
    C4: the spectra build 0.27 -> 0.20 ms per step (profiles/r04ab2_basis_gen_prefetch.txt)."""
    m = log2_exact(n)
    d = len(gen.z)
    on = force or os.environ.get("FGP_SPEC_BASIS_GEN", "1")[:1] != "0"
    if not on or not (17 <= m <= 24) or d > 6 or len(set(int(a) for a in gen.alphas)) != 1:
        return None
    Q = spec_chunks(LATTICE, n)
    wbytes = _spec_work_bytes(LATTICE, m, d)
    work = torch.empty((wbytes,), dtype=torch.uint8, device=device)
    out = torch.empty((Q, 2 ** d, 64), dtype=torch.float64, device=device)
    N.call("fgp_spec_basis_gen", N.int64_array(gen.z), m, int(d), 2 * int(gen.alphas[0]),
           N.double_array([lattice_coefficient(a) for a in gen.alphas]), N.ptr(out), N.ptr(work), wbytes,
           N.stream_ptr(device))
    return out


class FusedMLL(object):
    def __init__(self, family, parts, ysq, raw_scale, raw_lengthscales, raw_noise, logdet_weight, mll_const,
                 requires_grad=(True, True, False), lr=0.1, max_iters=1, parts_per_problem=False, per_problem=None,
                 gen=None, basis=None, mt=None, loss_metric="MLL", cv_weight=1.0):
        """
        family: 0 lattice (FFT) / 1 net (FWHT)
        basis:  part-product spectra (spec_basis) [Q, 2^d, 64] shared or [G, Q, 2^d, 64]: the spectral fit path
                (one kernel per iteration, no transform; parts / gen are then not used)
        parts:  [d, n] shared, or [G, d, n] when parts_per_problem; None with `gen` (LatticePartsGen)
        ysq:    [G, n]
        per_problem: the G problems are independent GPs with their own loss / Rprop (default: G == 1);
                otherwise one loss sums over the G problems (per-output hyper-parameters of one GP)
        raw_scale [S] with S in {1, G}; raw_lengthscales [S_l, D_l] with S_l in {1, G}, D_l in {1, d};
        raw_noise [S_n] with S_n in {1, G}
        mt:     multitask spectral fit (include/fgp_hip.h mt_tasks; G = 1, ysq only gives n): dict with
                `basis` the pair spectra [T (T+1)/2, 2^d, n], `ytilde` [T, n], `kt` the task kernel [T, T]
        loss_metric: "MLL" (default), or "GCV" / "CV" (fgp_nll_desc.loss_metric, ABI 16: the spectral path only;
                multitask: GCV ABI 17, CV ABI 18; cv_weight the scalar cv_weights of AbstractGP.fit); their loss
                history holds [loss, numer, denom] (CV: [loss, nan, nan])
        """
        if loss_metric != "MLL" and basis is None and mt is None:
            raise ValueError("GCV / CV fits run on the spectral path only (basis, or the multitask spectra)")
        require_device(ysq, "FusedMLL")
        self.device = ysq.device
        self.family = int(family)
        G, n = ysq.shape
        self.G, self.n = int(G), int(n)
        self.m = log2_exact(n)
        if self.m < 4:
            raise ValueError("fused fit needs n >= 16")
        if mt is not None:
            d = int(round(math.log2(mt["basis"].shape[1])))
            parts, gen, basis = None, None, None
        elif basis is not None:
            d = int(round(math.log2(basis.shape[-2])))
            parts, gen = None, None
        else:
            d = parts.shape[-2] if parts is not None else len(gen.z)
        self.d = int(d)
        if d > 8:
            raise ValueError("fused fit supports d <= 8")
        self.gen = gen
        self.basis = basis.contiguous() if basis is not None else None
        self.parts = parts.contiguous() if parts is not None else None
        if gen is not None and gen.shift.shape[0] not in (1, G):
            raise ValueError("generator shift rows must be 1 or G")
        self.ysq = ysq.contiguous()
        S = raw_scale.numel()
        Sl, Dl = raw_lengthscales.shape
        Sn = raw_noise.numel()
        for cnt in (S, Sl, Sn):
            if cnt not in (1, G):
                raise ValueError("hyper-parameter batch must be 1 or G")
        if Dl not in (1, d):
            raise ValueError("lengthscales last dim must be 1 or d")
        self.layout = dict(scale_off=0, scale_pp=int(S == G and G > 1),
                           ls_off=S, ls_pp=int(Sl == G and G > 1), ls_pd=int(Dl == d and Dl > 1 or d == 1),
                           noise_off=S + Sl * Dl, noise_pp=int(Sn == G and G > 1))
        if d == 1:
            self.layout["ls_pd"] = 1
        self.sizes = (S, Sl * Dl, Sn)
        self.n_params = S + Sl * Dl + Sn
        self.raw = torch.cat([raw_scale.reshape(-1), raw_lengthscales.reshape(-1), raw_noise.reshape(-1)]).to(
            device=self.device, dtype=torch.float64).contiguous()
        tk = mt.get("task") if mt is not None else None
        self.task = None
        if tk is not None:
            # a learned task kernel (ABI 18, GCV / CV): raw = [scale, lengthscales, noise, F [T][R], task noise [T]]
            fr = tk["factor"].detach().to(device=self.device, dtype=torch.float64)
            vr = tk["noise"].detach().to(device=self.device, dtype=torch.float64).reshape(-1)
            T, R = fr.shape
            self.task = dict(T=int(T), R=int(R), off=self.n_params, rg=tuple(bool(r) for r in tk["rg"]),
                             vexp=bool(tk["vexp"]))
            self.raw = torch.cat([self.raw, fr.reshape(-1), vr]).contiguous()
            self.n_params += int(T) * (int(R) + 1)
        cdt = torch.complex128 if self.family == 0 else torch.float64
        self.work = torch.empty((G, n), dtype=cdt, device=self.device) if (self.m > 12 and basis is None and
                                                                           mt is None) else None
        # Rprop state (previous gradient, step sizes), the gradient and the loss / parameter histories in ONE
        # zeroed allocation (one fill kernel + the step sizes' fill: a graph-replayed small fit pays per node)
        self.per_problem = bool(G == 1 if per_problem is None else per_problem)
        hmax = max(int(max_iters), 16)                  # ensure_history's first size
        hg = self.G if self.per_problem else 1
        np_ = self.n_params
        blob = torch.zeros((3 * np_ + hmax * hg * 3 + hmax * np_,), dtype=torch.float64, device=self.device)
        st = blob[:3 * np_].view(3, np_)
        st[1].fill_(float(lr))
        self.prev, self.step, self.grad = st[0], st[1], st[2]
        self._rprop_state = st[:2]                      # (prev, step) adjacent: refill resets both with one copy
        self.loss_hist = blob[3 * np_:3 * np_ + hmax * hg * 3].view(hmax, hg, 3)
        self.raw_hist = blob[3 * np_ + hmax * hg * 3:].view(hmax, np_)
        self.max_iters = hmax
        self._init_max_iters = max_iters
        self._nll = N.NllDesc(
            family=self.family, log2n=self.m, d=self.d, G=self.G,
            parts=(self.parts.data_ptr() if self.parts is not None else 0),
            parts_stride=(d * n if parts_per_problem else 0),
            ysq=self.ysq.data_ptr(), ysq_stride=n, raw=self.raw.data_ptr(),
            logdet_weight=float(logdet_weight),
            grad_lam=0, work=(self.work.data_ptr() if self.work is not None else 0),
            partials=0, **self.layout)
        self.loss_metric = loss_metric
        self._nll.loss_metric = {"MLL": N.LOSS_MLL, "GCV": N.LOSS_GCV, "CV": N.LOSS_CV}[loss_metric]
        self._nll.cv_weight = float(cv_weight)
        if gen is not None:
            gen.apply(self._nll, n)
        self.ysq_rows = self.ysq
        if self.basis is not None:
            self._nll.basis = self.basis.data_ptr()
            self._nll.basis_stride = self.basis[0].numel() if self.basis.dim() == 4 else 0
            # Y in the spectra's chunk layout [Q][G][64] (include/fgp_hip.h ysq_chunked): a chunk's spectra
            # and every problem's Y of it are two contiguous runs
            Q = spec_chunks(self.family, n)
            w = min(n, Q * 64)
            if w == Q * 64:                              # no padding: one copy (G = 1) or the transposing copy
                yp = self.ysq[:, :w].clone() if G == 1 else self.ysq[:, :w]
            else:
                yp = torch.zeros((G, Q * 64), dtype=torch.float64, device=self.device)
                yp[:, :w] = self.ysq[:, :w]
            self.ysq = yp.view(G, Q, 64).transpose(0, 1).contiguous()
            self._nll.ysq = self.ysq.data_ptr()
            self._nll.ysq_chunked = 1
        self.mt = None
        if mt is not None:
            T = int(mt["ytilde"].shape[0])
            self.mt = dict(basis=mt["basis"].contiguous(), ytilde=mt["ytilde"].contiguous(),
                           kt=mt["kt"].to(device=self.device, dtype=torch.float64).contiguous())
            assert tuple(self.mt["basis"].shape) == (T * (T + 1) // 2, 1 << d, n)
            self._nll.mt_tasks = T
            self._nll.mt_basis = self.mt["basis"].data_ptr()
            self._nll.mt_ytilde = self.mt["ytilde"].data_ptr()
            self._nll.mt_kt = self.mt["kt"].data_ptr()
            if self.task is not None:
                rg = self.task["rg"]
                self._nll.mt_task_rg = int(rg[0]) | (int(rg[1]) << 1)
                self._nll.mt_rank = self.task["R"]
                self._nll.mt_vexp = int(self.task["vexp"])
        plen = ctypes.c_int64(0)
        N.call("fgp_nll_partials_len", self._nll, ctypes.byref(plen))
        self.partials = torch.empty((plen.value,), dtype=torch.float64, device=self.device)
        self._nll.partials = self.partials.data_ptr()
        self.requires_grad = tuple(int(bool(r)) for r in requires_grad)
        self.mll_const = float(mll_const)
        self._fit = None
        self._refresh_fit_desc()
        self.ensure_history(self._init_max_iters)

    def ensure_history(self, iters):
        if iters <= self.max_iters:
            return
        new_max = max(iters, 2 * self.max_iters, 16)
        lh = torch.zeros((new_max, self.G if self.per_problem else 1, 3), dtype=torch.float64, device=self.device)
        rh = torch.zeros((new_max, self.n_params), dtype=torch.float64, device=self.device)
        if self.loss_hist is not None:
            lh[:self.max_iters] = self.loss_hist
            rh[:self.max_iters] = self.raw_hist
        self.loss_hist, self.raw_hist, self.max_iters = lh, rh, new_max
        self._refresh_fit_desc()

    def _refresh_fit_desc(self):
        if not hasattr(self, "mll_const"):
            return
        self._fit = N.FitDesc(
            n_params=self.n_params, raw=self.raw.data_ptr(), rprop_prev=self.prev.data_ptr(),
            rprop_step=self.step.data_ptr(), grad_out=self.grad.data_ptr(), loss_hist=self.loss_hist.data_ptr(),
            raw_hist=self.raw_hist.data_ptr(), scale_rg=self.requires_grad[0], ls_rg=self.requires_grad[1],
            noise_rg=self.requires_grad[2], mll_const=self.mll_const, eta_minus=RPROP_ETAS[0],
            eta_plus=RPROP_ETAS[1], step_min=RPROP_STEPS[0], step_max=RPROP_STEPS[1],
            per_problem=int(self.per_problem))

    def stream(self):
        return N.stream_ptr(self.device)

    def run(self, iter0, iters, final_no_update=False):
        """Enqueue `iters` fit iterations writing history rows iter0 .. iter0+iters-1.

        Independent problems (per_problem, G >= 2) can run as `groups()` problem groups, each driven by
        fgp_fit_run on its own HIP stream (sub-descriptors over a problem range, joined back to the
        current stream by events), meant to overlap one group's VALU-bound row kernels with another
        group's HBM-bound column kernel (measured slower, see groups()).  Every problem's arithmetic is
        the same as in the single launch sequence (bit-identical results)."""
        self.ensure_history(iter0 + iters)
        self._raw_entry = None
        groups = self.groups()
        if groups <= 1:
            if iters >= FIT_GRAPH_MIN_ITERS and os.environ.get("FGP_FIT_GRAPH", "1")[:1] != "0":
                # the launch sequence replayed from a hipGraph of this engine (fgp_fit_run_graph, ABI 17): the
                # replayed per-launch rate, bit-identical results; short runs (the early-stopping loop's first chunks)
                # stay eager, a capture per call would not pay
                N.call("fgp_fit_run_graph", self._nll, self._fit, int(iter0), int(iters), int(bool(final_no_update)),
                       self._graph_token(), self.stream())
                return
            N.call("fgp_fit_run", self._nll, self._fit, int(iter0), int(iters), int(bool(final_no_update)),
                   self.stream())
            return
        subs = self._group_descs(groups)
        cur = torch.cuda.current_stream(self.device)
        start = torch.cuda.Event()
        start.record(cur)
        for (nll, fit, _), st in zip(subs, self._streams):
            st.wait_event(start)
            N.call("fgp_fit_run", nll, fit, int(iter0), int(iters), int(bool(final_no_update)), st.cuda_stream)
        for st in self._streams[:groups]:
            done = torch.cuda.Event()
            done.record(st)
            cur.wait_event(done)

    def refill(self, ysq, raw_scale, raw_lengthscales, raw_noise, lr, basis):
        """Reuse this engine for a new fit of the same geometry (cached_engine): the new Y in the engine's own buffer,
        the initial raw parameters, a fresh Rprop state (torch.optim.Rprop's: prev 0, step lr), the fit's spectra
        (at the address the descriptors hold).  Histories are rewritten row by row by the fit."""
        assert basis.data_ptr() == self._nll.basis
        self.basis = basis
        G, n = ysq.shape
        if self._nll.ysq_chunked:
            Q = spec_chunks(self.family, n)
            w = min(n, Q * 64)
            if w == Q * 64:
                self.ysq.copy_(ysq[:, :w].view(G, Q, 64).transpose(0, 1))
            else:
                yp = torch.zeros((G, Q * 64), dtype=torch.float64, device=self.device)
                yp[:, :w] = ysq[:, :w]
                self.ysq.copy_(yp.view(G, Q, 64).transpose(0, 1))
        else:
            self.ysq.copy_(ysq)
        self.ysq_rows = ysq
        src = [raw_scale.reshape(-1), raw_lengthscales.reshape(-1), raw_noise.reshape(-1)]
        torch.cat(src, out=self.raw)
        # run_persist's entry state (a barrier give-up restores it): the caller's tensors themselves, not a copy (the
        # fit replaces a GP's Parameters by new ones, abstract_gp.py:295-296, it never writes into them)
        self._raw_entry = src
        init = getattr(self, "_rprop_init", None)      # [[0 ...], [lr ...]] on the device, kept per lr
        if init is None or init[0] != float(lr):
            t = torch.zeros_like(self._rprop_state)
            t[1].fill_(float(lr))
            init = self._rprop_init = (float(lr), t)
        self._rprop_state.copy_(init[1])

    def release_inputs(self):
        """Drop the references to the fit's inputs (spectra, Y rows) after the fit is enqueued: a cached engine must not
        keep the caller's spectra alive (the next fit's spectra could then not take their address)."""
        self.basis = None
        self.ysq_rows = None

    def _graph_token(self):
        """This engine's token for fgp_fit_run_graph's cache (released when the engine is freed)."""
        tok = getattr(self, "_token", None)
        if tok is None:
            global _NEXT_TOKEN
            _NEXT_TOKEN += 1
            tok = self._token = _NEXT_TOKEN
        return tok

    def __del__(self):
        tok = getattr(self, "_token", None)
        if tok is not None:
            try:
                N.call("fgp_fit_graph_release", tok)
            except Exception:
                pass

    def persist_ok(self):
        """fgp_fit_persist applies (one problem on the spectral path whose spectra fit the LDS of at most 64
        workgroups: the whole fit in one launch); FGP_FIT_PERSIST=0 keeps the launch per iteration."""
        return self.persist_workgroups() > 0

    def persist_workgroups(self):
        """Workgroups of the single-launch fit (fgp_fit_persist_ok: 0 outside its domain, or when they would not
        all be co-resident on this device)."""
        if os.environ.get("FGP_FIT_PERSIST", "1")[:1] == "0" or self.G != 1 or not self._nll.basis:
            return 0
        wg = getattr(self, "_persist_wg", None)      # (a function of the engine's geometry and the device only)
        if wg is None:
            ok = ctypes.c_int(0)
            N.call("fgp_fit_persist_ok", self._nll, ctypes.byref(ok))
            wg = self._persist_wg = ok.value
        return wg

    def run_persist(self, iterations, logtol, wait_max, defer=False):
        """AbstractGP.fit's iterations 0 .. iterations with its early-stopping rule, in one launch
        (fgp_fit_persist); returns the last iteration evaluated (its row applied no update).  Afterwards `raw` holds
        the BEST iterate's parameters (ABI 18), the ones AbstractGP.fit restores.

        The 4-int control word is read back at once (one small device-to-host read), or with `defer` by
        persist_result() once the caller has enqueued its own work behind the launch (-1 is returned): when an
        in-kernel barrier gave up (the workgroups were not co-resident after all -- e.g. CUs taken by other work), the
        entry parameters are restored (the kernel leaves Rprop's state untouched and sets the parameters to NaN) and
        None is returned, so the caller re-runs the fit on the launch per iteration, which gives the same trajectory
        bit for bit.  Inside a hipGraph capture nothing can be read: the word is kept for check_persist at the next
        eager call, and a failure shows as NaN parameters and parameter history."""
        self.check_persist()
        self.ensure_history(iterations + 1)
        ctrl = torch.empty((4,), dtype=torch.int32, device=self.device)   # (the launch clears the words it reports)
        capturing = torch.cuda.is_current_stream_capturing()
        entry, self._raw_entry = getattr(self, "_raw_entry", None), None
        raw0 = None if capturing else (entry if entry is not None else self.raw.clone())
        N.call("fgp_fit_persist", self._nll, self._fit, int(iterations), float(logtol), int(wait_max),
               ctrl.data_ptr(), self.stream())
        if capturing:
            self._ctrl = ctrl
            return int(iterations)
        self._pending = (ctrl, raw0)
        return -1 if defer else self.persist_result()

    def persist_result(self):
        """The control word of the last run_persist: its last iteration, or None after a barrier give-up (the entry
        parameters restored); synchronises."""
        ctrl, raw0 = self._pending
        self._pending = None
        c = ctrl.cpu().tolist()
        if c[2]:
            if isinstance(raw0, list):
                torch.cat(raw0, out=self.raw)
            else:
                self.raw.copy_(raw0)
            self.persist_failures = getattr(self, "persist_failures", 0) + 1
            return None
        return int(c[1])

    def check_persist(self):
        """Raise for a failed fgp_fit_persist whose control word could not be read when it ran (a capture)."""
        ctrl = getattr(self, "_ctrl", None)
        if ctrl is None:
            return None
        self._ctrl = None
        c = ctrl.cpu().tolist()
        if c[2]:
            raise RuntimeError("fgp_fit_persist: an in-kernel barrier gave up (workgroups not co-resident?)")
        return int(c[1])

    def groups(self):
        """Problem groups of run(): FGP_FIT_STREAMS (default 1) for independent problems, else 1.
        Measured on MI355X (8 GPs, n = 2^20, profiles/r02e_exp_fit_streams.jsonl): 1 group 93.6 us per
        iteration, 2 groups 136 us, 4 groups 100 us -- the side-stream launches do not overlap usefully,
        so the single launch sequence is the default."""
        if not self.per_problem or self.G < 2:
            return 1
        try:
            k = int(os.environ.get("FGP_FIT_STREAMS", "1"))
        except ValueError:
            k = 1
        return max(1, min(k, self.G, 4))

    def _group_descs(self, groups):
        """(nll, fit, partials) sub-descriptors of problem ranges [G k / groups, G (k+1) / groups)."""
        key = (groups, self._fit.loss_hist, self._fit.raw_hist)
        if getattr(self, "_groups_key", None) == key:
            return self._groups
        if getattr(self, "_streams", None) is None or len(self._streams) < groups:
            self._streams = [torch.cuda.Stream(self.device) for _ in range(groups)]
        G, n, d = self.G, self.n, self.d
        out = []
        for k in range(groups):
            g0, g1 = G * k // groups, G * (k + 1) // groups
            Gk = g1 - g0
            nll = N.NllDesc()
            ctypes.pointer(nll)[0] = self._nll
            nll.G = Gk
            nll.ysq = self.ysq_rows[g0].data_ptr()      # row layout for a problem range
            nll.ysq_chunked = 0
            plen = ctypes.c_int64(0)
            N.call("fgp_nll_partials_len", nll, ctypes.byref(plen))
            part = torch.empty((plen.value,), dtype=torch.float64, device=self.device)
            if self.work is not None:
                nll.work = self.work[g0].data_ptr()
            nll.partials = part.data_ptr()
            if self.parts is not None and self._nll.parts_stride:
                nll.parts = self.parts[g0].data_ptr()
            if self.gen is not None and self._nll.gen_shift_stride:
                nll.gen_shift = self.gen.shift[g0].data_ptr()
            if self.basis is not None and self._nll.basis_stride:
                nll.basis = self.basis[g0].data_ptr()
            lay = self.layout
            dl = self.sizes[1] // (G if lay["ls_pp"] else 1)
            if lay["scale_pp"]:
                nll.scale_off = lay["scale_off"] + g0
            if lay["ls_pp"]:
                nll.ls_off = lay["ls_off"] + g0 * dl
            if lay["noise_pp"]:
                nll.noise_off = lay["noise_off"] + g0
            for name, flag in (("scale_pp", lay["scale_pp"]), ("ls_pp", lay["ls_pp"]), ("noise_pp", lay["noise_pp"])):
                setattr(nll, name, int(flag and Gk > 1))
            fit = N.FitDesc()
            ctypes.pointer(fit)[0] = self._fit
            fit.hist_stride = G
            fit.hist_offset = g0
            out.append((nll, fit, part))
        self._groups_key, self._groups = key, out
        return out

    def evaluate(self, slot=0):
        """Loss terms and gradient at the current raw parameters (no update); synchronises."""
        self.ensure_history(slot + 1)
        self._raw_entry = None
        st = self.stream()
        N.call("fgp_nll_fwd", self._nll, st)
        N.call("fgp_nll_bwd", self._nll, st)
        N.call("fgp_fit_step", self._nll, self._fit, int(slot), 0, st)
        lh = self.loss_hist[slot].sum(0).cpu() if self.per_problem else self.loss_hist[slot, 0].cpu()
        return float(lh[0]), float(lh[1]), float(lh[2]), self.grad.cpu()

    def fit_step(self, slot, update=True):
        """Enqueue the reduction + Rprop step of history slot `slot` (fgp_fit_step)."""
        self.ensure_history(slot + 1)
        self._raw_entry = None
        N.call("fgp_fit_step", self._nll, self._fit, int(slot), int(bool(update)), self.stream())

    def stage(self, k):
        """Enqueue one kernel of the fwd/bwd pipeline (fgp_nll_stage; per-kernel timing)."""
        N.call("fgp_nll_stage", self._nll, int(k), self.stream())

    def split_raw(self, raw_vec):
        S, L, Nn = self.sizes
        return raw_vec[..., :S], raw_vec[..., S:S + L], raw_vec[..., S + L:S + L + Nn]

    def split_task(self, raw_vec):
        """(raw task factor [.., T R], raw task noise [.., T]) of a learned task kernel's raw vector(s); None without."""
        if self.task is None:
            return None
        o, T, R = self.task["off"], self.task["T"], self.task["R"]
        return raw_vec[..., o:o + T * R], raw_vec[..., o + T * R:o + T * (R + 1)]

    def task_kernel_rows(self, raw_rows):
        """K_task = F F^T + diag(v) of every history row (util.py:157-162); None without a learned task kernel."""
        if self.task is None:
            return None
        f, v = self.split_task(raw_rows)
        T, R = self.task["T"], self.task["R"]
        F = f.reshape(f.shape[:-1] + (T, R))
        vv = torch.exp(v) if self.task["vexp"] else v
        return torch.einsum("...il,...kl->...ik", F, F) + torch.diag_embed(vv)


_ENGINES = collections.OrderedDict()
ENGINE_CACHE_SIZE = 4


def cached_engine(family, ysq, raw_scale, raw_lengthscales, raw_noise, logdet_weight, mll_const, requires_grad, lr,
                  max_iters, basis, per_problem=None, loss_metric="MLL", cv_weight=1.0):
    """The FusedMLL of a spectral fit, reused across fit() calls of the same geometry (LRU of ENGINE_CACHE_SIZE): its
    buffers keep their addresses, so fgp_fit_run_graph replays the engine's captured launch sequence instead of
    capturing anew, and the host builds no engine per call (fit() at the replayed rate).  The spectra
    must be at the same address (a rebuilt set usually is: the freed one's block).  FGP_ENGINE_CACHE=0: a new engine
    per call."""
    G, n = ysq.shape
    S, (Sl, Dl), Sn = raw_scale.numel(), raw_lengthscales.shape, raw_noise.numel()
    key = (str(ysq.device), int(family), int(G), int(n), basis.data_ptr(), tuple(basis.shape), S, Sl, Dl, Sn,
           per_problem, float(logdet_weight), float(mll_const), tuple(bool(r) for r in requires_grad), int(max_iters),
           loss_metric, float(cv_weight))
    on = os.environ.get("FGP_ENGINE_CACHE", "1")[:1] != "0"
    eng = _ENGINES.get(key) if on else None
    if eng is not None:
        _ENGINES.move_to_end(key)
        eng.refill(ysq, raw_scale, raw_lengthscales, raw_noise, lr, basis)
        return eng
    eng = FusedMLL(family, None, ysq, raw_scale, raw_lengthscales, raw_noise, logdet_weight=logdet_weight,
                   mll_const=mll_const, requires_grad=requires_grad, lr=lr, max_iters=max_iters,
                   per_problem=per_problem, basis=basis, loss_metric=loss_metric, cv_weight=cv_weight)
    if on:
        _ENGINES[key] = eng
        while len(_ENGINES) > ENGINE_CACHE_SIZE:
            _ENGINES.popitem(last=False)
    return eng


def persist_giveups(reset=False):
    """The library's sticky count of single-launch-fit barrier give-ups (fgp_persist_giveups, ABI 17; synchronises)."""
    c = ctypes.c_ulonglong(0)
    N.call("fgp_persist_giveups", ctypes.byref(c), int(bool(reset)))
    return int(c.value)


def check_replayed_fits(before):
    """Raise when a single-launch fit gave up since the count `before` (persist_giveups()) was read: after hipGraph
    replays of captured fits, whose control words the capture could not read -- such a fit's parameters are NaN, not
    a result (fit_engine.FusedMLL.run_persist)."""
    now = persist_giveups()
    if now != before:
        raise RuntimeError("fgp_fit_persist: %d in-kernel barrier give-up(s) during replayed fits (their parameters are "
                           "NaN; workgroups not co-resident?)" % (now - before))
    return now


def mll_constant(d_out, n):
    """d_out * n * log(2 pi) (fastgps/abstract_gp.py:235)."""
    return d_out * n * math.log(2 * math.pi)


def spec_inv_eig(family, raw_scale, raw_lengthscales, raw_noise, G, n, basis):
    """A = 1/ev [G, n] float64 (ev = sqrt(n) lambda + noise, lambda = scale sum_S l^S Phi_S real) of G
    problems from part-product spectra `basis` ([Q, 2^d, 64] shared or [G, Q, 2^d, 64]) via fgp_spec_inv_eig
    -- fgp_inv_eig's wa without materialising lambda."""
    require_device(basis, "spec_inv_eig")
    d, dev = int(round(math.log2(basis.shape[-2]))), basis.device
    m = log2_exact(n)
    S, (Sl, Dl), Sn = raw_scale.numel(), raw_lengthscales.shape, raw_noise.numel()
    raw = torch.cat([raw_scale.reshape(-1), raw_lengthscales.reshape(-1), raw_noise.reshape(-1)]).to(
        device=dev, dtype=torch.float64).contiguous()
    wa = torch.empty((G, n), dtype=torch.float64, device=dev)
    basis = basis.contiguous()
    desc = N.NllDesc(family=family, log2n=m, d=d, G=G, parts=0, parts_stride=0, ysq=wa.data_ptr(), ysq_stride=0,
                     raw=raw.data_ptr(), scale_off=0, scale_pp=int(S == G and G > 1), ls_off=S,
                     ls_pp=int(Sl == G and G > 1), ls_pd=int(Dl == d), noise_off=S + Sl * Dl,
                     noise_pp=int(Sn == G and G > 1), logdet_weight=1.0, grad_lam=0, work=0, partials=wa.data_ptr(),
                     basis=basis.data_ptr(), basis_stride=(basis[0].numel() if basis.dim() == 4 else 0))
    N.call("fgp_spec_inv_eig", desc, N.ptr(wa), N.stream_ptr(dev))
    return wa


def _spec_desc(family, raw, S, Sl, Dl, Sn, G, n, d, basis, scratch):
    m = log2_exact(n)
    return N.NllDesc(family=family, log2n=m, d=d, G=G, parts=0, parts_stride=0, ysq=scratch.data_ptr(), ysq_stride=0,
                     raw=raw.data_ptr(), scale_off=0, scale_pp=int(S == G and G > 1), ls_off=S,
                     ls_pp=int(Sl == G and G > 1), ls_pd=int(Dl == d), noise_off=S + Sl * Dl,
                     noise_pp=int(Sn == G and G > 1), logdet_weight=1.0, grad_lam=0, work=0,
                     partials=scratch.data_ptr(), basis=basis.data_ptr(),
                     basis_stride=(basis[0].numel() if basis.dim() == 4 else 0))


def spec_post_var(raw_scale, raw_lengthscales, raw_noise, G, n, basis, psi, part0):
    """Posterior variances [G, N] of G lattice problems sharing the part-product spectra `basis` ([Q, 2^d, 64])
    at N test points from the row spectra psi [N, 2^d, n] (complex128, fftbr of the part-product rows of
    each test point) via fgp_spec_post_var: ft(K_g(x_t, .)) = scale_g sum_S l_g^S psi[t, S] by linearity."""
    require_device(basis, "spec_post_var")
    d, dev = int(round(math.log2(basis.shape[-2]))), basis.device
    Nt = psi.shape[0]
    assert psi.shape == (Nt, 2 ** d, n) and psi.dtype == torch.complex128 and psi.is_contiguous()
    S, (Sl, Dl), Sn = raw_scale.numel(), raw_lengthscales.shape, raw_noise.numel()
    raw = torch.cat([raw_scale.reshape(-1), raw_lengthscales.reshape(-1), raw_noise.reshape(-1)]).to(
        device=dev, dtype=torch.float64).contiguous()
    nblk = (n // 2 + 1 + 1023) // 1024
    partial = torch.empty((max(1, G * Nt * nblk),), dtype=torch.float64, device=dev)
    out = torch.empty((G, Nt), dtype=torch.float64, device=dev)
    basis = basis.contiguous()
    desc = _spec_desc(0, raw, S, Sl, Dl, Sn, G, n, d, basis, partial)
    N.call("fgp_spec_post_var", desc, N.ptr(psi), Nt, N.double_array([float(v) for v in part0]), N.ptr(out),
           N.ptr(partial), N.stream_ptr(dev))
    return out


def fused_lam(family, parts, raw_scale, raw_lengthscales, raw_noise, G, gen=None, n=None, basis=None):
    """lambda = ft(k1) for G eigen-problems sharing `parts` ([d, n]), with parts of their own
    ([G, d, n]), with the generator `gen` (size n), or from part-product spectra `basis` ([Q, 2^d, 64]
    shared, [G, Q, 2^d, 64]), via fgp_nll_lam -> [G, n]."""
    parts_stride = 0
    if basis is not None:
        require_device(basis, "fused_lam")
        d, dev = int(round(math.log2(basis.shape[-2]))), basis.device
        parts, gen = None, None
    elif parts is not None:
        require_device(parts, "fused_lam")
        d, n = parts.shape[-2:]
        dev = parts.device
        parts = parts.contiguous()
        if parts.dim() == 3:
            assert parts.shape[0] == G
            parts_stride = d * n
    else:
        require_device(gen.shift, "fused_lam")
        d, dev = len(gen.z), gen.shift.device
    m = log2_exact(n)
    S, (Sl, Dl), Sn = raw_scale.numel(), raw_lengthscales.shape, raw_noise.numel()
    raw = torch.cat([raw_scale.reshape(-1), raw_lengthscales.reshape(-1), raw_noise.reshape(-1)]).to(
        device=dev, dtype=torch.float64).contiguous()
    cdt = torch.complex128 if family == 0 else torch.float64
    out = torch.empty((G, n), dtype=cdt, device=dev)
    work = torch.empty((G, n), dtype=cdt, device=dev) if (m > 12 and basis is None) else None
    desc = N.NllDesc(family=family, log2n=m, d=d, G=G, parts=(parts.data_ptr() if parts is not None else 0),
                     parts_stride=parts_stride,
                     ysq=out.data_ptr(), ysq_stride=0, raw=raw.data_ptr(),
                     scale_off=0, scale_pp=int(S == G and G > 1), ls_off=S, ls_pp=int(Sl == G and G > 1),
                     ls_pd=int(Dl == d), noise_off=S + Sl * Dl, noise_pp=int(Sn == G and G > 1), logdet_weight=1.0,
                     grad_lam=out.data_ptr(), work=(work.data_ptr() if work is not None else 0),
                     partials=out.data_ptr())
    if gen is not None:
        gen.apply(desc, n)
    if basis is not None:
        basis = basis.contiguous()
        desc.basis = basis.data_ptr()
        desc.basis_stride = basis[0].numel() if basis.dim() == 4 else 0
    N.call("fgp_nll_lam", desc, N.stream_ptr(dev))
    return out
