"""Multitask and derivative-informed FastGPLattice / FastGPDigitalNetB2 on MI355X.

`FastGPLattice(..., num_tasks=T)` / `FastGPDigitalNetB2(..., num_tasks=T)` with T > 1, or with
`derivatives=` / `derivatives_coeffs=`, construct these classes (fast_gp.py routes them), mirroring the
reference's multitask semantics (abstract_gp.py:45-150 construction, :152-306 fit, :307-474 data and
predictions; abstract_fast_gp.py:29-31,155-191 task-pair caches and derivative kernel parts; util.py:
40-62, 95-183, 275-394 caches and the block inverse).

Where the work runs:
  * derivative kernel parts, per task pair and for prediction rows  -> fgp_mt_parts (HIP)
  * ft / ift of every task's data and first-column kernels           -> fgp_fftbr / fgp_ifftbr / fgp_fwht
  * the T x T block-eigenvalue inverse (util.py:275-337), its solves,
    logdet and the MLL gradient                                      -> fgp_mt_factor / fgp_mt_solve /
                                                                       fgp_mt_selinv / fgp_mt_mll_grad
  * kernel-from-parts products, the task kernel F F^T + diag(v), the packing of the eigenvalue
    blocks and the optimizer step: torch ops on the device (autograd carries the hyper-parameter
    gradients through them and through the HIP transforms).
The GCV / CV losses and predictions requested WITH an autograd graph use a dense per-frequency-class
statement of the same blocks (torch.linalg on the device) -- they need gradients of functionals of
the whole inverse that the structured kernels do not provide.  There is no CPU fallback.
"""
import ctypes
import math
import os

import numpy as np
import torch

from . import ops
from . import _native as N
from .fast_gp import _IDENTITY_TFS, AbstractFastGP, _Hyper, _as_size, _exp, _identity
from .fit_engine import RPROP_ETAS, RPROP_STEPS, FusedMLL, mll_constant


def _to_n_tensor(n):
    if isinstance(n, (int, np.integer)):
        return torch.tensor([int(n)], dtype=torch.int64)
    if isinstance(n, (list, tuple)):
        return torch.tensor([int(v) for v in n], dtype=torch.int64)
    assert isinstance(n, torch.Tensor)
    return n.detach().to("cpu", torch.int64).reshape(-1)


class _Layout(object):
    """Sorted active tasks of an n-vector (util.py:273-274) and the packed block layout."""

    def __init__(self, ns):
        self.ns = [int(v) for v in ns]
        self.task_order = torch.tensor(self.ns).argsort(descending=True).tolist()   # the reference's call
        self.active = [o for o in self.task_order if self.ns[o] > 0]
        self.nsrt = [self.ns[o] for o in self.active]
        self.T = len(self.active)
        assert self.T >= 1, "cannot build the inverse without data"
        self.nmin = self.nsrt[-1]
        self.R = sum(v // self.nmin for v in self.nsrt)
        self.lay = ops.mt_layout(self.nsrt)
        self.pairs = [(k, l) for k in range(self.T) for l in range(k, self.T)]
        self.off = {}
        L = 0
        for (k, l) in self.pairs:
            self.off[k, l] = L
            L += self.nsrt[k]
        self.L = L
        self.rs = [sum(v // self.nmin for v in self.nsrt[:k]) for k in range(self.T)]

    def pack(self, vecs):
        """per-task vectors (task order) [..., n_l] -> [..., R nmin] (sorted, concatenated)."""
        return torch.cat([vecs[o] for o in self.active], -1)

    def unpack(self, v, like_batch):
        parts = v.split(self.nsrt, -1)
        out = [None] * len(self.ns)
        for i, o in enumerate(self.active):
            out[o] = parts[i]
        for o in range(len(self.ns)):
            if out[o] is None:
                out[o] = torch.zeros(tuple(like_batch) + (0,), dtype=v.dtype, device=v.device)
        return out

    def dense_index(self, device):
        """(positions in the packed array, row, col) of every pattern entry, for the dense statement."""
        pos, rows, cols = [], [], []
        for (k, l) in self.pairs:
            qk, ql = self.nsrt[k] // self.nmin, self.nsrt[l] // self.nmin
            for q in range(qk):
                base = self.off[k, l] + q * self.nmin
                pos.append(torch.arange(base, base + self.nmin))
                rows.append(torch.full((self.nmin,), self.rs[k] + q, dtype=torch.int64))
                cols.append(torch.full((self.nmin,), self.rs[l] + q % ql, dtype=torch.int64))
        jj = torch.arange(self.nmin).repeat(len(pos))
        return (torch.cat(pos).to(device), torch.cat(rows).to(device), torch.cat(cols).to(device), jj.to(device))


class MultiTaskFastGP(AbstractFastGP):
    """num_tasks > 1 and / or derivative-informed fast GP (shared by both families; the family class
    supplies ft / ift / get_omega and the point conversion)."""

    _MULTITASK = True

    def __init__(self, seqs, num_tasks, seed_for_seq, alpha, scale, lengthscales, noise, factor_task_kernel,
                 rank_factor_task_kernel, noise_task_kernel, device, tfs_scale, tfs_lengthscales, tfs_noise,
                 tfs_factor_task_kernel, tfs_noise_task_kernel, requires_grad_scale, requires_grad_lengthscales,
                 requires_grad_noise, requires_grad_factor_task_kernel, requires_grad_noise_task_kernel, shape_batch,
                 shape_scale, shape_lengthscales, shape_noise, shape_factor_task_kernel, shape_noise_task_kernel,
                 derivatives, derivatives_coeffs, compile_fts, compile_fts_kwargs, adaptive_nugget,
                 data_dtype=torch.float64):
        torch.nn.Module.__init__(self)
        assert torch.get_default_dtype() == torch.float64, \
            "fast transforms do not work without torch.float64 precision"
        assert data_dtype == torch.float64, "multitask / derivative-informed GPs run in float64 (the reference's)"
        self.data_dtype = torch.float64
        if num_tasks is None:
            self.solo_task, self.default_task, num_tasks = True, 0, 1
        else:
            assert isinstance(num_tasks, int) and num_tasks > 0
            self.solo_task, self.default_task = False, torch.arange(num_tasks)
        T = self.num_tasks = num_tasks
        assert T <= ops.N.MT_MAX_TASKS, "at most %d tasks" % ops.N.MT_MAX_TASKS
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("fastgaussianprocesses_amd runs on a HIP device (device='cuda'); got %s" % device)
        dev = self.device
        self.seqs = self._resolve_seqs(seqs, seed_for_seq, T)
        self.seq = self.seqs[0]
        self.d = int(self.seqs[0].d)
        assert all(int(s.d) == self.d for s in self.seqs)
        d = self.d
        self.n = torch.zeros(T, dtype=torch.int64, device=dev)
        self.m = -torch.ones(T, dtype=torch.int64, device=dev)
        self._ns = [0] * T
        # derivatives (abstract_gp.py:58-72)
        if derivatives is not None or derivatives_coeffs is not None:
            rank_factor_task_kernel = 1
            tfs_noise_task_kernel = _IDENTITY_TFS
            noise_task_kernel = 0.
        if derivatives is None:
            derivatives = [torch.zeros((1, d), dtype=torch.int64, device=dev) for _ in range(T)]
        if isinstance(derivatives, torch.Tensor):
            derivatives = [derivatives]
        assert isinstance(derivatives, list) and len(derivatives) == T
        derivatives = [v[None, :] if v.ndim == 1 else v for v in derivatives]
        assert all(v.ndim == 2 and v.size(1) == d for v in derivatives)
        self.derivatives = [v.to(device=dev, dtype=torch.int64) for v in derivatives]
        self._derivs_h = [v.detach().cpu().to(torch.int64) for v in derivatives]
        if derivatives_coeffs is None:
            derivatives_coeffs = [torch.ones(len(v), device=dev) for v in self.derivatives]
        assert isinstance(derivatives_coeffs, list) and len(derivatives_coeffs) == T
        assert all(c.ndim == 1 and len(c) == len(v) for c, v in zip(derivatives_coeffs, self.derivatives))
        self.derivatives_coeffs = [c.to(device=dev, dtype=torch.float64) for c in derivatives_coeffs]
        # shapes and hyper-parameters (abstract_gp.py:73-139)
        shape_batch = _as_size(shape_batch)
        assert isinstance(shape_batch, torch.Size)
        self.shape_batch = shape_batch
        self.ndim_batch = len(shape_batch)
        scale = _Hyper.make(scale, shape_scale, shape_batch, lambda v: v == 1, "scale", "pos", dev)
        if shape_lengthscales is None and not isinstance(lengthscales, torch.Tensor):
            shape_lengthscales = torch.Size([d])
        lengthscales = _Hyper.make(lengthscales, shape_lengthscales, shape_batch, lambda v: v in (1, d),
                                   "lengthscales", "pos", dev)
        noise = _Hyper.make(noise, shape_noise, shape_batch, lambda v: v == 1, "noise", "pos", dev)
        if shape_factor_task_kernel is None and not isinstance(factor_task_kernel, torch.Tensor):
            if rank_factor_task_kernel is None:
                rank_factor_task_kernel = 0 if T == 1 else 1
            assert isinstance(rank_factor_task_kernel, int) and 0 <= rank_factor_task_kernel <= T
            shape_factor_task_kernel = torch.Size([T, rank_factor_task_kernel])
        factor_task_kernel = _Hyper.make(factor_task_kernel, shape_factor_task_kernel, shape_batch,
                                         lambda v: 0 <= v <= T, "factor_task_kernel", None, dev, core=2)
        assert factor_task_kernel.shape[-2] == T
        if shape_noise_task_kernel is None and not isinstance(noise_task_kernel, torch.Tensor):
            shape_noise_task_kernel = torch.Size([T])
        noise_task_kernel = _Hyper.make(noise_task_kernel, shape_noise_task_kernel, shape_batch,
                                        lambda v: v in (T, 1), "noise_task_kernel", "nonneg", dev)
        for tfs in (tfs_scale, tfs_lengthscales, tfs_noise, tfs_factor_task_kernel, tfs_noise_task_kernel):
            assert len(tfs) == 2 and callable(tfs[0]) and callable(tfs[1]), \
                "tfs should be a tuple of two callables, the transform and inverse transform"
        self._tfs = dict(scale=tfs_scale, lengthscales=tfs_lengthscales, noise=tfs_noise)
        self.tf_scale, self.tf_lengthscales, self.tf_noise = tfs_scale[1], tfs_lengthscales[1], tfs_noise[1]
        self.tf_factor_task_kernel, self.tf_noise_task_kernel = tfs_factor_task_kernel[1], tfs_noise_task_kernel[1]
        if requires_grad_factor_task_kernel is None:
            requires_grad_factor_task_kernel = T > 1
        if requires_grad_noise_task_kernel is None:
            requires_grad_noise_task_kernel = T > 1
        self.raw_scale = torch.nn.Parameter(tfs_scale[0](scale), requires_grad=requires_grad_scale)
        self.raw_lengthscales = torch.nn.Parameter(tfs_lengthscales[0](lengthscales),
                                                   requires_grad=requires_grad_lengthscales)
        self.raw_noise = torch.nn.Parameter(tfs_noise[0](noise), requires_grad=requires_grad_noise)
        self.raw_factor_task_kernel = torch.nn.Parameter(tfs_factor_task_kernel[0](factor_task_kernel),
                                                         requires_grad=bool(requires_grad_factor_task_kernel))
        self.raw_noise_task_kernel = torch.nn.Parameter(tfs_noise_task_kernel[0](noise_task_kernel),
                                                        requires_grad=bool(requires_grad_noise_task_kernel))
        # derivative multitask setting checks (abstract_gp.py:146-150)
        self._deriv_mode = any(bool((v > 0).any()) for v in self._derivs_h) or \
            any(bool((c != 1).any()) for c in self.derivatives_coeffs)
        if self._deriv_mode:
            self.raw_noise_task_kernel.requires_grad_(False)
            self.raw_factor_task_kernel.requires_grad_(False)
            assert (self.gram_matrix_tasks == 1).all()
        self.adaptive_nugget = adaptive_nugget
        self.compile_fts, self.compile_fts_kwargs = compile_fts, compile_fts_kwargs
        # alpha (abstract_fast_gp.py:21-24)
        assert (np.isscalar(alpha) and alpha % 1 == 0) or (isinstance(alpha, torch.Tensor) and alpha.shape == (d,)), \
            "alpha should be an int or a torch.Tensor of length d"
        if np.isscalar(alpha):
            alpha = int(alpha) * torch.ones(d, dtype=torch.int64, device=dev)
        self.alpha = alpha
        self._alphas = [int(a) for a in alpha.tolist()]
        self._family_checks()
        # storage
        self._y = [torch.empty(0, device=dev) for _ in range(T)]
        self._xs = [torch.empty((0, d), device=dev) for _ in range(T)]
        self._xbs = [torch.empty((0, d), dtype=self._XBDTYPE, device=dev) for _ in range(T)]
        self._pts = [0] * T
        self._yt_state = [None] * T
        self._parts_cache = {}
        self._cache = {}
        self._snap = None

    # ------------------------------------------------------------------ sequences and points
    def _resolve_seqs(self, seqs, seed_for_seq, T):
        if isinstance(seqs, (int, np.integer)):
            return [self._default_seq(int(seqs), s) for s in np.random.SeedSequence(seed_for_seq).spawn(T)]
        if not isinstance(seqs, (list, tuple, np.ndarray)):
            seqs = [seqs]
        seqs = list(seqs)
        assert len(seqs) == T, "seqs should be a length num_tasks=%d list" % T
        for s in seqs:
            self._check_seq(s)
        return seqs

    def _family_checks(self):
        if self._FAMILY == ops.NET:
            ts = [int(s.t) for s in self.seqs]
            assert all(t < 64 for t in ts), "each seq must have t<64"
            assert all(t == ts[0] for t in ts), "all seqs should have the same t"
            self.t = ts[0]
            if self.num_tasks > 1:
                assert all(getattr(s, "randomize", "DS") in ["FALSE", "DS"] for s in self.seqs), \
                    "each seq should have randomize in ['FALSE','DS']"
            assert all(1 <= a <= 4 for a in self._alphas)
            if any(bool((v != 0).any()) for v in self._derivs_h):
                assert all(a >= 2 for a in self._alphas), "using derivatives requires (alpha>=2).all()"

    def _sample_task(self, l, n_min, n_max):
        return self._sample_seq(self.seqs[l], n_min, n_max)      # the family's generator (device when own)

    def _ensure_task_points(self, l, n):
        n = int(n)
        if n <= self._pts[l]:
            return
        x, xb = self._sample_task(l, self._pts[l], n)
        self._xs[l] = torch.cat([self._xs[l], x], 0)
        self._xbs[l] = self._xs[l] if self._FAMILY == ops.LATTICE else torch.cat([self._xbs[l], xb], 0)
        self._pts[l] = n

    def get_x(self, task, n=None):
        assert 0 <= task < self.num_tasks
        n = self._ns[task] if n is None else int(n)
        assert n >= 0
        self._ensure_task_points(task, n)
        return self._xs[task][:n]

    def get_xb(self, task, n=None):
        assert 0 <= task < self.num_tasks
        n = self._ns[task] if n is None else int(n)
        assert n >= 0
        self._ensure_task_points(task, n)
        return self._xbs[task][:n]

    def _task_list(self, task):
        if task is None:
            task = self.default_task
        inttask = isinstance(task, int)
        if inttask:
            task = torch.tensor([task], dtype=torch.int64)
        if isinstance(task, list):
            task = torch.tensor(task, dtype=torch.int64)
        assert task.ndim == 1 and (task >= 0).all() and (task < self.num_tasks).all()
        return inttask, [int(v) for v in task.tolist()]

    def get_x_next(self, n, task=None):
        """abstract_fast_gp.py:32-37 + abstract_gp.py:310-330."""
        if isinstance(n, (int, np.int64)):
            nt = torch.tensor([n], dtype=torch.int64)
        elif isinstance(n, list):
            nt = torch.tensor(n, dtype=torch.int64)
        else:
            nt = n.detach().cpu().to(torch.int64)
        assert isinstance(nt, torch.Tensor) and torch.logical_or(nt == 0, nt & (nt - 1) == 0).all(), \
            "maximum sequence index must be a power of 2"
        inttask, tasks = self._task_list(task)
        assert nt.ndim == 1 and len(nt) == len(tasks)
        assert all(int(nt[i]) >= self._ns[l] for i, l in enumerate(tasks)), \
            "maximum sequence index must be greater than the current number of samples"
        out = [self.get_x(l, int(nt[i]))[self._ns[l]:] for i, l in enumerate(tasks)]
        return out[0] if inttask else out

    def add_y_next(self, y_next, task=None):
        """abstract_gp.py:331-351 + abstract_fast_gp.py:38-40."""
        if isinstance(y_next, torch.Tensor):
            y_next = [y_next]
        inttask, tasks = self._task_list(task)
        assert isinstance(y_next, list) and len(y_next) == len(tasks)
        assert all(y.shape[:-1] == self.shape_batch for y in y_next)
        for y, l in zip(y_next, tasks):
            st = self._yt_state[l]
            if st is None or self._ns[l] == 0 or st[0] > self._ns[l]:
                self._yt_state[l] = None        # only an append keeps the cached prefix transform valid
            self._y[l] = torch.cat([self._y[l], y.to(device=self.device, dtype=torch.float64)], -1)
        self._ns = [int(y.size(-1)) for y in self._y]
        self.n = torch.tensor(self._ns, dtype=torch.int64, device=self.device)
        self.m = torch.tensor([v.bit_length() - 1 if v > 0 else -1 for v in self._ns], dtype=torch.int64,
                              device=self.device)
        self._cache = {}
        assert all(v == 0 or (v & (v - 1)) == 0 for v in self._ns), "total samples must be power of 2"

    @property
    def x(self):
        xs = [self.get_x(l) for l in range(self.num_tasks)]
        return xs[0] if self.solo_task else xs

    @property
    def y(self):
        return self._y[0] if self.solo_task else self._y

    # ------------------------------------------------------------------ hyper-parameters
    @property
    def gram_matrix_tasks(self):
        """F F^T + diag(noise_task_kernel) (util.py:157-162)."""
        F = self.factor_task_kernel
        k = torch.einsum("...il,...kl->...ik", F, F)
        return k + self.noise_task_kernel[..., None] * torch.eye(self.num_tasks, device=self.device)

    def _fused_ok(self):
        return False

    # ------------------------------------------------------------------ fused multitask fit
    def _mt_fused_ok(self):
        """The device-resident multitask MLL fit (k_mt_spec_iter + the spectral reduction / Rprop step,
        include/fgp_hip.h mt_tasks) covers: every task with the same n >= 16, at most 8 tasks, d <= 6, no
        parameter batch, the task kernel fixed (derivative-informed GPs fix it at 1, abstract_gp.py:146-150),
        exp parameter transforms, no adaptive nugget.  FGP_MT_FUSED=0 takes the generic autograd loop."""
        if os.environ.get("FGP_MT_FUSED", "1")[:1] == "0" or os.environ.get("FGP_MT_GENERAL", "0")[:1] == "1":
            return False
        ns = self._ns
        n = ns[0]
        if not (n >= 16 and all(v == n for v in ns) and self.num_tasks <= 8 and self.d <= 6):
            return False
        if self.adaptive_nugget or len(self.shape_batch) or self.raw_factor_task_kernel.requires_grad or \
                self.raw_noise_task_kernel.requires_grad:
            return False
        if any(self._tfs[k][1] is not _exp for k in ("scale", "lengthscales", "noise")):
            return False
        T = self.num_tasks
        if (T * (T + 1) // 2) * (1 << self.d) * n * 16 > MT_SPECTRA_CAP:
            return False
        return tuple(self.raw_scale.shape) == (1,) and tuple(self.raw_noise.shape) == (1,) and \
            tuple(self.raw_lengthscales.shape) in ((1,), (self.d,))

    def _mt_learn_ok(self):
        """fit(loss_metric="GCV" / "CV") on the device with the task kernel LEARNED (ABI 18: k_mt_spec_iter's LEARN
        variants + k_mt_learn_step; the reference's default for num_tasks > 1, abstract_gp.py:116-139): _mt_fused_ok's
        domain except the fixed task kernel -- the factor [T, R] with the identity transform, the task noise [T] with the
        exp or the identity transform, no parameter batch."""
        if os.environ.get("FGP_MT_FUSED", "1")[:1] == "0":
            return False
        if not (self.raw_factor_task_kernel.requires_grad or self.raw_noise_task_kernel.requires_grad):
            return False
        ns = self._ns
        n, T = ns[0], self.num_tasks
        if not (n >= 16 and all(v == n for v in ns) and 2 <= T <= 8 and self.d <= 6):
            return False
        if self.adaptive_nugget or len(self.shape_batch):
            return False
        if any(self._tfs[k][1] is not _exp for k in ("scale", "lengthscales", "noise")):
            return False
        if self.tf_factor_task_kernel is not _identity or self.tf_noise_task_kernel not in (_exp, _identity):
            return False
        if tuple(self.raw_factor_task_kernel.shape[:-1]) != (T,) or tuple(self.raw_noise_task_kernel.shape) != (T,):
            return False
        if (T * (T + 1) // 2) * (1 << self.d) * n * 16 > MT_SPECTRA_CAP:
            return False
        return tuple(self.raw_scale.shape) == (1,) and tuple(self.raw_noise.shape) == (1,) and \
            tuple(self.raw_lengthscales.shape) in ((1,), (self.d,))

    def _mt_param_rows(self):
        """Parameter batches (docs/examples/batch_multitask/fgp_lattice.ipynb cell 6; abstract_gp.py:73-139: each
        parameter's batch dimensions are the TRAILING dimensions of shape_batch): None when no parameter has batch
        dimensions (one problem, the data batch sharing the parameters), else the [5, d_out] int tensor of every
        output's row in each parameter block (scale, lengthscales, noise, task factor, task noise) and the blocks'
        row counts -- each output its own eigen-problem (fgp_mt_fit_desc.G / rows, ABI 16)."""
        tails = ((self.raw_scale, 1), (self.raw_lengthscales, 1), (self.raw_noise, 1), (self.raw_factor_task_kernel, 2),
                 (self.raw_noise_task_kernel, 1))
        bshapes = [tuple(p.shape[:p.dim() - t]) for p, t in tails]
        if not any(bshapes):
            return None
        sb = tuple(int(v) for v in self.shape_batch)
        d_out = int(np.prod(sb)) if sb else 1
        grid = np.stack(np.meshgrid(*[np.arange(v) for v in sb], indexing="ij"), -1).reshape(d_out, len(sb)) \
            if sb else np.zeros((1, 0), dtype=np.int64)
        rows, nrows = [], []
        for bs in bshapes:
            k = len(bs)
            if k > len(sb) or tuple(sb[len(sb) - k:]) != bs:
                return False
            sub = grid[:, len(sb) - k:]
            rows.append(np.ravel_multi_index(tuple(sub.T), bs) if k else np.zeros(d_out, dtype=np.int64))
            nrows.append(int(np.prod(bs)) if k else 1)
        return np.stack(rows).astype(np.int32), nrows

    def _mt_general_ok(self):
        """The device-resident fit of the GENERAL case (fgp_mt_fit_run, ABI 14: MtGeneralEngine) -- the reference's
        default multitask setting (abstract_gp.py:116-139: the task kernel F F^T + diag(v) learned), any n per
        task (util.py:273-323), a data batch sharing the hyper-parameters or (ABI 16) parameter batches broadcast
        over shape_batch (every output its own eigen-problem, at most 4096): at most 16 active tasks, d <= 6, exp
        transforms for scale / lengthscales / noise, the identity for the task factor and exp or the identity for
        the task noise (one per task), the plain or (ABI 16) the adaptive nugget, pair spectra within MT_SPECTRA_CAP
        bytes."""
        if os.environ.get("FGP_MT_FUSED", "1")[:1] == "0":
            return False
        lo_ns = [v for v in self._ns if v > 0]
        if not lo_ns or self.d > 6 or len(lo_ns) > N.MT_MAX_TASKS:
            return False
        if any(self._tfs[k][1] is not _exp for k in ("scale", "lengthscales", "noise")):
            return False
        if self.tf_factor_task_kernel is not _identity or self.tf_noise_task_kernel not in (_exp, _identity):
            return False
        T = self.num_tasks
        if self.raw_scale.shape[-1] != 1 or self.raw_noise.shape[-1] != 1 or \
                self.raw_lengthscales.shape[-1] not in (1, self.d) or self.raw_factor_task_kernel.dim() < 2 or \
                self.raw_factor_task_kernel.shape[-2] != T or self.raw_noise_task_kernel.shape[-1] != T:
            return False
        pr = self._mt_param_rows()
        if pr is False or (pr is not None and (len(pr[0][0]) > 4096 or
                                              sum(n * w for n, w in zip(pr[1], self._mt_row_widths())) > 8192)):
            return False
        srt = sorted(lo_ns, reverse=True)
        spec = sum(srt[k] for k in range(len(srt)) for _ in range(k, len(srt))) * (1 << self.d) * 16
        return spec <= MT_SPECTRA_CAP

    def _mt_row_widths(self):
        """Raw elements per row of each parameter block (scale, lengthscales, noise, task factor, task noise)."""
        return (1, int(self.raw_lengthscales.shape[-1]), 1,
                int(self.raw_factor_task_kernel.shape[-1]) * self.num_tasks, self.num_tasks)

    def _mt_spectra(self, n):
        """Pair spectra Phi^{kl}_S = ft(B^{kl}_S) [T (T+1)/2, 2^d, n] (pairs k <= l row-major): with the
        derivative parts of get_k1parts(k, l) (abstract_fast_gp.py:173-180) and _kernel_from_parts'
        k1_kl = scale sum_{b0, b1} c0 c1 prod_j (ind_j + l_j parts_j) (:181-191) expanded over the subsets S of
        the dimensions, B^{kl}_S = sum over the (b0, b1) whose derivative dimensions lie in S of
        c0 c1 prod_{j in S} parts_j -- so lam_kl = ft(k1_kl) = scale sum_S l^S Phi^{kl}_S (ft linear)."""
        def f():
            T, d, dev = self.num_tasks, self.d, self.device
            NS = 1 << d
            ins = torch.tensor([[bool((S >> j) & 1) for j in range(d)] for S in range(NS)])   # [NS, d]
            insd = ins.to(dev)
            rows = []
            for k in range(T):
                for l in range(k, T):
                    parts = self.get_k1parts(k, l, n)                         # [n, p0, p1, d]
                    b0, b1 = self._derivs_h[k], self._derivs_h[l]
                    need = (b0[:, None, :] + b1[None, :, :]) > 0              # [p0, p1, d]
                    valid = (~need[None] | ins[:, None, None, :]).all(-1)    # [NS, p0, p1]
                    cc = self.derivatives_coeffs[k][:, None] * self.derivatives_coeffs[l][None, :]
                    # prod_{j in S} parts_j for every subset at once (ascending j), [NS, n, p0, p1]
                    prod = torch.where(insd[:, None, None, None, :], parts[None], 1.0).prod(-1)
                    w = cc[None] * valid.to(device=dev, dtype=torch.float64)                 # [NS, p0, p1]
                    rows.append((prod * w[:, None]).sum((-1, -2)))           # [NS, n]
            B = torch.stack(rows)                                            # [T (T+1) / 2, NS, n]
            return self.ft(B).contiguous()
        return self._cached(("mt_spec", n), f, grad_sensitive=False)

    def _pair_spectra(self, lo):
        """Spectra of the sorted pairs of the general engine (fgp_mt_fit_desc.spectra): for sorted pair
        (k, l), tasks a = active[k], b = active[l], the reference's lam_kl is get_lam(a, b, n_k) for a <= b and
        get_lam(b, a, n_k).conj() otherwise (util.py:280-284), so Phi^{kl}_S = ft(B_S) (conjugated for a > b),
        B_S the part products of get_k1parts(min, max, n_k) as in _mt_spectra.  Returns (flat complex128
        tensor, offsets of every pair in complex elements)."""
        def f():
            d, dev = self.d, self.device
            NS = 1 << d
            ins = torch.tensor([[bool((S >> j) & 1) for j in range(d)] for S in range(NS)])
            insd = ins.to(dev)
            Bs, conj, offs, off = [], [], [], 0
            for (k, l) in lo.pairs:
                a, b = lo.active[k], lo.active[l]
                t0, t1 = (a, b) if a <= b else (b, a)
                nk = lo.nsrt[k]
                parts = self.get_k1parts(t0, t1, nk)                              # [nk, p0, p1, d]
                if not self._deriv_mode:
                    # no derivatives (one (b0, b1) = (0, 0) term, coefficient 1): B_S = prod_{j in S} parts_j -- the
                    # same values as the weighted sum below (x * 1.0, one-term sums), without its host-side mask copy
                    B = torch.where(insd[:, None, :], parts[None, :, 0, 0, :], 1.0).prod(-1)   # [NS, nk]
                else:
                    b0, b1 = self._derivs_h[t0], self._derivs_h[t1]
                    need = (b0[:, None, :] + b1[None, :, :]) > 0
                    valid = (~need[None] | ins[:, None, None, :]).all(-1)
                    cc = self.derivatives_coeffs[t0][:, None] * self.derivatives_coeffs[t1][None, :]
                    prod = torch.where(insd[:, None, None, None, :], parts[None], 1.0).prod(-1)
                    w = cc[None] * valid.to(device=dev, dtype=torch.float64)
                    B = (prod * w[:, None]).sum((-1, -2))                        # [NS, nk]
                Bs.append(B)
                conj.append(a > b)
                offs.append(off)
                off += NS * nk
            # one transform per distinct n over the pairs of that length (rows are transformed independently: the
            # same values as pair by pair)
            specs = [None] * len(Bs)
            for nk in sorted(set(int(B.shape[-1]) for B in Bs)):
                idx = [i for i, B in enumerate(Bs) if int(B.shape[-1]) == nk]
                ft = self.ft(torch.cat([Bs[i] for i in idx])).to(torch.complex128)
                for r, i in enumerate(idx):
                    sp = ft[r * NS:(r + 1) * NS]
                    specs[i] = (sp.conj() if conj[i] else sp).resolve_conj().reshape(-1)
            return torch.cat(specs).contiguous(), offs
        return self._cached(("mt_pair_spec", tuple(lo.nsrt), tuple(lo.active)), f, grad_sensitive=False)

    def _fused_engine(self, iterations, lr, ysq=None, d_out=None, loss_metric="MLL", cv_weight=1.0):
        """FusedMLL in multitask spectral mode (G = 1; loss_metric MLL, GCV (ABI 17) or CV (ABI 18)); the general
        engine (MtGeneralEngine, MLL) outside its domain (_mt_fused_ok: equal n, fixed task kernel)."""
        learn = loss_metric != "MLL" and not self._mt_fused_ok() and self._mt_learn_ok()
        if not self._mt_fused_ok() and not learn:
            return MtGeneralEngine(self, lr, min(iterations + 1, 64))
        n, T = self._ns[0], self.num_tasks
        yt = torch.stack([self.get_ytilde(k).reshape(n) for k in range(T)])
        ls = self.raw_lengthscales.detach()
        mt = dict(basis=self._mt_spectra(n), ytilde=yt, kt=self.gram_matrix_tasks.detach())
        if learn:
            # the task kernel's parameters in the engine's raw vector (FusedMLL: K_task formed on the device)
            mt["task"] = dict(factor=self.raw_factor_task_kernel, noise=self.raw_noise_task_kernel,
                              rg=(self.raw_factor_task_kernel.requires_grad, self.raw_noise_task_kernel.requires_grad),
                              vexp=self.tf_noise_task_kernel is _exp)
        return FusedMLL(self._FAMILY, None, torch.zeros((1, n), device=self.device),
                        self.raw_scale.detach().reshape(-1), ls.reshape(1, -1), self.raw_noise.detach().reshape(-1),
                        logdet_weight=1.0, mll_const=mll_constant(1, T * n),
                        requires_grad=(self.raw_scale.requires_grad, self.raw_lengthscales.requires_grad,
                                       self.raw_noise.requires_grad),
                        lr=lr, max_iters=min(iterations + 1, 64), loss_metric=loss_metric, cv_weight=cv_weight, mt=mt)

    # ------------------------------------------------------------------ kernel parts and kernels
    # (_pair_spec, _kargs, _parts_pairs, _kernel_from_parts: AbstractFastGP, fast_gp.py)
    def _kmat_block(self, x, z, ta, tb, zip_pairs=False, chunk_elems=1 << 24):
        """K_{ta,tb}(x_i, z_k) -> [*param batch, N, M] ([*, N] with zip_pairs), chunked over x."""
        b0, b1 = self._derivs_h[ta], self._derivs_h[tb]
        c0, c1 = self.derivatives_coeffs[ta], self.derivatives_coeffs[tb]
        bd0, bd1 = self.derivatives[ta], self.derivatives[tb]
        N = x.shape[0]
        per = max(1, (1 if zip_pairs else z.shape[0]) * len(b0) * len(b1) * self.d)
        step = max(1, chunk_elems // per)
        outs = []
        for i0 in range(0, N, step):
            xs = x[i0:i0 + step]
            zs = z[i0:i0 + step] if zip_pairs else z
            p = self._parts_pairs(xs, zs, b0, b1, zip_pairs)
            outs.append(self._kernel_from_parts(p, bd0, bd1, c0, c1))
        if not outs:
            shape = (0,) if zip_pairs else (0, z.shape[0])
            return self._kernel_from_parts(torch.zeros(shape + (len(b0), len(b1), self.d), device=self.device),
                                           bd0, bd1, c0, c1)
        return torch.cat(outs, -1 if zip_pairs else -2)

    def get_k1parts(self, task0, task1, n=None):
        """_K1PartsSeq[task0, task1][:n] (util.py:50-62): points of task0 vs the first point of task1."""
        assert 0 <= task0 < self.num_tasks and 0 <= task1 < self.num_tasks
        n = self._ns[task0] if n is None else int(n)
        assert n >= 0
        key = (task0, task1, n)
        if key not in self._parts_cache:
            xa = self.get_xb(task0, n)
            zb = self.get_xb(task1, 1)
            self._parts_cache[key] = self._parts_pairs(xa, zb, self._derivs_h[task0], self._derivs_h[task1],
                                                       check=False)[:, 0]
        return self._parts_cache[key]

    def get_lam(self, task0, task1, n=None):
        """_LamCaches[task0, task1] (util.py:95-132, abstract_fast_gp.py:155-160): ft of the first-column
        kernel at n points of task0 (task0 <= task1)."""
        assert 0 <= task0 < self.num_tasks and 0 <= task1 < self.num_tasks
        assert task0 <= task1, "lam caches exist for task0 <= task1 (abstract_fast_gp.py:30)"
        n = self._ns[task0] if n is None else int(n)

        def k1_of(parts):
            return self._kernel_from_parts(parts, self.derivatives[task0], self.derivatives[task1],
                                           self.derivatives_coeffs[task0], self.derivatives_coeffs[task1])

        def f():
            half = self._cache.get(("lam", (task0, task1, n // 2), True, False)) \
                if (n >= 4 and not self._gradmode()) else None
            if half is not None:
                # _LamCaches doubling (util.py:113-132): one DIT stage from the cached lam at n/2 and ft
                # of the first-column kernel over the new half of task0's points
                new = self._parts_pairs(self.get_xb(task0, n)[n // 2:], self.get_xb(task1, 1),
                                        self._derivs_h[task0], self._derivs_h[task1], check=False)[:, 0]
                return ops.double_update(self._FAMILY, half, self.ft(k1_of(new)))
            return self.ft(k1_of(self.get_k1parts(task0, task1, n)))
        return self._cached(("lam", (task0, task1, n)), f)

    def get_ytilde(self, task):
        """_YtildeCache (util.py:164-183)."""
        assert 0 <= task < self.num_tasks
        n = self._ns[task]

        def f():
            y = self._y[task]
            st = self._yt_state[task]
            if st is not None and 1 < st[0] < n and n % st[0] == 0:
                ns, yt = st                     # _YtildeCache doubling (util.py:173-178)
                while ns < n:
                    yt = ops.double_update(self._FAMILY, yt, self.ft(y[..., ns:2 * ns]))
                    ns *= 2
            else:
                yt = self.ft(y) if n > 1 else y.clone().to(self._FTOUTDTYPE)
            self._yt_state[task] = (n, yt)
            return yt
        return self._cached(("ytilde", (task, n)), f, grad_sensitive=False)

    # ------------------------------------------------------------------ the block inverse
    def _nvec(self, n):
        if n is None:
            return list(self._ns)
        nt = _to_n_tensor(n)
        assert nt.shape == (self.num_tasks,), "n must hold one size per task"
        assert all(int(v) >= c for v, c in zip(nt.tolist(), self._ns))
        return [int(v) for v in nt.tolist()]

    def _lams_blocks(self, lo):
        """The reference's lams[k, l] (util.py:277-298) for the sorted active tasks, packed [*G, L]."""
        Kt = self.gram_matrix_tasks
        lams = {}
        for (k, l) in lo.pairs:
            a, b = lo.active[k], lo.active[l]
            lam = self.get_lam(a, b, lo.nsrt[k]) if a <= b else self.get_lam(b, a, lo.nsrt[k]).conj()
            lams[k, l] = math.sqrt(lo.nsrt[l]) * lam.to(torch.complex128)
        noise = self.noise
        if self.adaptive_nugget:
            i0 = lo.active.index(0) if 0 in lo.active else 0
            tr00 = lams[i0, i0].sum(-1, keepdim=True)
            for k in range(lo.T):
                lams[k, k] = lams[k, k] + noise * (lams[k, k].sum(-1, keepdim=True) / tr00).abs()
        else:
            for k in range(lo.T):
                lams[k, k] = lams[k, k] + noise
        for (k, l) in lo.pairs:
            lams[k, l] = lams[k, l] * Kt[..., lo.active[k], lo.active[l], None]
        bshape = torch.broadcast_shapes(*[lams[kl].shape[:-1] for kl in lo.pairs])
        packed = torch.cat([lams[kl].expand(bshape + lams[kl].shape[-1:]) for kl in lo.pairs], -1)
        return packed, bshape

    def _factor(self, ns):
        """(layout, factor [G, L], logdet [*G], G, Gshape) without an autograd graph (cached)."""
        def f():
            lo = _Layout(ns)
            with torch.no_grad():
                packed, gshape = self._lams_blocks(lo)
                G = int(np.prod(gshape)) if len(gshape) else 1
                fac, ld, info = ops.mt_factor(lo.lay, packed.reshape(G, lo.L))
            return lo, fac, ld.sum(-1).reshape(gshape), G, gshape
        return self._cached(("mt_factor", tuple(ns)), f)

    def _selinv(self, ns):
        def f():
            lo, fac, _, G, gshape = self._factor(ns)
            return ops.mt_selinv(lo.lay, fac)
        return self._cached(("mt_selinv", tuple(ns)), f)

    def _dense_inverse(self, ns):
        """Differentiable dense statement: Lambda_j [*G, nmin, R, R] -> (A [*G, R, R, nmin], logdet [*G])."""
        lo = _Layout(ns)
        packed, gshape = self._lams_blocks(lo)
        pos, rows, cols, jj = lo.dense_index(self.device)
        flat = packed.reshape((-1, lo.L))
        G = flat.shape[0]
        M = torch.zeros((G, lo.nmin, lo.R, lo.R), dtype=torch.complex128, device=self.device)
        vals = flat[:, pos]
        M = M.index_put((torch.arange(G, device=self.device)[:, None], jj[None, :], rows[None, :], cols[None, :]),
                        vals)
        off = rows != cols
        Mlow = torch.zeros_like(M).index_put((torch.arange(G, device=self.device)[:, None], jj[None, off],
                                              cols[None, off], rows[None, off]), vals[:, off].conj())
        M = M + Mlow
        A = torch.linalg.inv(M)
        logdet = torch.linalg.slogdet(M).logabsdet.sum(-1)
        return lo, A.permute(0, 2, 3, 1).reshape(tuple(gshape) + (lo.R, lo.R, lo.nmin)), logdet.reshape(gshape)

    def get_inv_log_det(self, n=None):
        """(inv [*G, R, R, nmin], logdet [*G]) as _FastInverseLogDetCache.__call__ (util.py:275-337)."""
        ns = self._nvec(n)
        if self._gradmode():
            _, A, logdet = self._dense_inverse(ns)
            return A, logdet
        lo, fac, logdet, G, gshape = self._factor(ns)

        def f():
            eye = torch.zeros((lo.R, G, lo.R, lo.nmin), dtype=torch.complex128, device=self.device)
            idx = torch.arange(lo.R, device=self.device)
            eye[idx, :, idx, :] = 1
            cols = ops.mt_solve(lo.lay, fac, eye.reshape(lo.R * G, lo.R * lo.nmin))
            A = cols.reshape(lo.R, G, lo.R, lo.nmin).permute(1, 2, 0, 3)
            if self._FAMILY == ops.NET:
                A = A.real
            return A.reshape(tuple(gshape) + (lo.R, lo.R, lo.nmin)).contiguous()
        return self._cached(("mt_inv_dense", tuple(ns)), f), logdet

    def _tilde_solve(self, vts, ns):
        """_gram_matrix_solve_tilde_to_tilde (util.py:354-363): per-task transformed vectors -> A v."""
        if self._gradmode():
            lo, A, _ = self._dense_inverse(ns)
            v = lo.pack([t.to(torch.complex128) for t in vts])
            v = v.reshape(v.shape[:-1] + (lo.R, lo.nmin))
            z = torch.einsum("...rcj,...cj->...rj", A.to(torch.complex128), v)
            return lo, lo.unpack(z.reshape(z.shape[:-2] + (-1,)), z.shape[:-2])
        lo, fac, _, G, gshape = self._factor(ns)
        v = lo.pack([t.to(torch.complex128) for t in vts])
        bshape = torch.broadcast_shapes(v.shape[:-1], tuple(gshape))
        v = v.expand(bshape + v.shape[-1:]).reshape(-1, v.shape[-1])
        z = ops.mt_solve(lo.lay, fac, v).reshape(bshape + (v.shape[-1],))
        return lo, lo.unpack(z, bshape)

    def gram_matrix_solve(self, y, n=None):
        """_FastInverseLogDetCache.gram_matrix_solve (util.py:338-353): y [..., sum n] in task order."""
        ns = self._nvec(n)
        assert y.size(-1) == sum(ns)
        ys = y.split(ns, dim=-1)
        vts = [self.ft(ys[l]) if ns[l] > 0 else ys[l].to(self._FTOUTDTYPE) for l in range(self.num_tasks)]
        lo, zs = self._tilde_solve(vts, ns)
        outs = []
        for l in range(self.num_tasks):
            z = zs[l]
            if ns[l] == 0:
                outs.append(z.real)
            elif self._FAMILY == ops.LATTICE:
                outs.append(self.ift(z).real)
            else:
                outs.append(self.ift(z.real))
        return torch.cat(outs, -1)

    @property
    def coeffs(self):
        """K^-1 y (util.py:396-425)."""
        return self._cached(("coeffs", tuple(self._ns)), lambda: self.gram_matrix_solve(torch.cat(self._y, -1)))

    # ------------------------------------------------------------------ losses and fit
    def _norm_logdet(self):
        """get_norm_term_logdet_term (util.py:364-370) through the HIP factor / solve / gradient."""
        ns = list(self._ns)
        lo = _Layout(ns)
        packed, gshape = self._lams_blocks(lo)
        G = int(np.prod(gshape)) if len(gshape) else 1
        Y = lo.pack([self.get_ytilde(l).to(torch.complex128) for l in range(self.num_tasks)])
        bshape = torch.broadcast_shapes(Y.shape[:-1], tuple(gshape))
        Yb = Y.expand(bshape + Y.shape[-1:]).reshape(-1, Y.shape[-1])
        norm, logdet = ops.mt_mll_terms(lo.lay, packed.reshape(G, lo.L), Yb)
        return norm.reshape(bshape + (1,)), logdet.reshape(tuple(gshape) + (1,))

    def _gcv_numer_denom(self):
        """get_gcv_numer_denom (util.py:371-380), dense statement (differentiable)."""
        ns = list(self._ns)
        lo, A, _ = self._dense_inverse(ns)
        Y = lo.pack([self.get_ytilde(l).to(torch.complex128) for l in range(self.num_tasks)])
        v = Y.reshape(Y.shape[:-1] + (lo.R, lo.nmin))
        z = torch.einsum("...rcj,...cj->...rj", A, v)
        numer = (z.conj() * z).real.sum((-1, -2))[..., None]
        idx = torch.arange(lo.R, device=self.device)
        tr = A[..., idx, idx, :].real.sum(-1).sum(-1, keepdim=True)
        denom = ((tr / sum(ns)) ** 2).real
        return numer, denom

    def _inv_diag(self):
        """get_inv_diag (util.py:381-394).  One task: the reference's mean(1 / (sqrt(n) lam)) (:382-385; real
        part on lattices, as the CV loss takes it).  Several: diag of K^-1 by solving the identity
        (O(n^2 log n)), its rows laid out [nsum, 1 per parameter-batch dim, nsum] so they broadcast against the
        hyper-parameter batch instead of pairing with it, then permuted batch-first (:387-393)."""
        if self.num_tasks == 1:
            lam = self.get_lam(0, 0)
            inv = (1 / (lam * math.sqrt(lam.size(-1)))).mean(-1, keepdim=True)
            return inv.real if inv.is_complex() else inv
        ns = list(self._ns)
        nsum = sum(ns)
        gshape = tuple(self._factor(ns)[4])
        nb = len(gshape)
        eye = torch.eye(nsum, device=self.device).reshape((nsum,) + (1,) * nb + (nsum,))
        kinv = self.gram_matrix_solve(eye)                    # [nsum, *batch, nsum]
        kinv = kinv.permute(tuple(range(1, kinv.ndim - 1)) + (0, kinv.ndim - 1))
        idx = torch.arange(nsum, device=self.device)
        return kinv[..., idx, idx]

    def fit(self, loss_metric="MLL", iterations=5000, lr=None, optimizer=None, stop_crit_improvement_threshold=5e-2,
            stop_crit_wait_iterations=10, store_hists=False, store_loss_hist=False, store_scale_hist=False,
            store_lengthscales_hist=False, store_noise_hist=False, store_task_kernel_hist=False, verbose=5,
            verbose_indent=4, masks=None, cv_weights=1):
        """abstract_gp.py:152-306 (every iteration recomputes the caches: FASTGP_FORCE_RECOMPILE)."""
        assert isinstance(loss_metric, str) and loss_metric.upper() in ["MLL", "GCV", "CV"]
        assert sum(self._ns) > 0, "cannot fit without data"
        assert isinstance(iterations, int) and iterations >= 0
        default_optimizer = optimizer is None
        if optimizer is None:
            optimizer = self.get_default_optimizer(lr)
        assert isinstance(optimizer, torch.optim.Optimizer)
        assert (isinstance(verbose, int) or isinstance(verbose, bool)) and verbose >= 0, \
            "require verbose is a non-negative int"
        assert isinstance(verbose_indent, int) and verbose_indent >= 0, \
            "require verbose_indent is a non-negative int"
        assert np.isscalar(stop_crit_improvement_threshold) and 0 < stop_crit_improvement_threshold, \
            "require stop_crit_improvement_threshold is a positive float"
        assert isinstance(stop_crit_wait_iterations, int) and stop_crit_wait_iterations > 0
        assert masks is None or isinstance(masks, torch.Tensor)
        loss_metric = loss_metric.upper()
        alt_dev = (loss_metric in ("GCV", "CV") and default_optimizer and masks is None and
                   (self._mt_fused_ok() or self._mt_learn_ok()) and os.environ.get("FGP_ALT_LOSS_DEVICE", "1")[:1] != "0")
        if loss_metric == "CV":
            # (one task: the reference's inv_diag is the single-task formula without the noise, util.py:383-386; a
            # per-point cv_weights needs the points' coefficients, not their Parseval sum)
            alt_dev = alt_dev and self.num_tasks > 1 and (
                np.isscalar(cv_weights) or (torch.is_tensor(cv_weights) and cv_weights.numel() == 1))
        if alt_dev:
            # GCV / CV of T tasks with equal n and a fixed task kernel (derivative-informed GPs) on the device:
            # k_mt_spec_iter's GCV / CV variants + k_spec_loss_step (ABI 17 / 18; util.py:371-394,
            # abstract_gp.py:242-272)
            hists = dict(loss=store_hists or store_loss_hist,
                         scale=store_hists or (store_scale_hist and self.raw_scale.requires_grad),
                         lengthscales=store_hists or (store_lengthscales_hist and self.raw_lengthscales.requires_grad),
                         noise=store_hists or (store_noise_hist and self.raw_noise.requires_grad),
                         task_kernel=store_hists or (store_task_kernel_hist and (
                             self.raw_factor_task_kernel.requires_grad or self.raw_noise_task_kernel.requires_grad)))
            return self._fit_fused(iterations, 1e-1 if lr is None else lr,
                                   (np.log(1 + stop_crit_improvement_threshold), stop_crit_wait_iterations), hists,
                                   verbose, verbose_indent, loss_metric=loss_metric,
                                   cv_weight=float(cv_weights) if loss_metric == "CV" else 1.0)
        if loss_metric == "MLL" and default_optimizer and masks is None and (self._mt_fused_ok() or
                                                                            self._mt_general_ok()):
            learned_tk = self.raw_factor_task_kernel.requires_grad or self.raw_noise_task_kernel.requires_grad
            hists = dict(loss=store_hists or store_loss_hist,
                         scale=store_hists or (store_scale_hist and self.raw_scale.requires_grad),
                         lengthscales=store_hists or (store_lengthscales_hist and self.raw_lengthscales.requires_grad),
                         noise=store_hists or (store_noise_hist and self.raw_noise.requires_grad),
                         task_kernel=store_hists or (store_task_kernel_hist and learned_tk))
            return self._fit_fused(iterations, 1e-1 if lr is None else lr,
                                   (np.log(1 + stop_crit_improvement_threshold), stop_crit_wait_iterations), hists,
                                   verbose, verbose_indent)
        logtol = np.log(1 + stop_crit_improvement_threshold)
        h_loss = store_hists or store_loss_hist
        h_scale = store_hists or (store_scale_hist and self.raw_scale.requires_grad)
        h_ls = store_hists or (store_lengthscales_hist and self.raw_lengthscales.requires_grad)
        h_noise = store_hists or (store_noise_hist and self.raw_noise.requires_grad)
        h_tk = store_hists or (store_task_kernel_hist and (self.raw_factor_task_kernel.requires_grad or
                                                           self.raw_noise_task_kernel.requires_grad))
        if masks is not None:
            masks = torch.atleast_2d(masks)
            assert masks.ndim == 2 and len(masks) <= len(self.shape_batch)
            d_out = torch.empty(self.shape_batch)[(..., *masks)].numel()
        else:
            d_out = int(torch.tensor(self.shape_batch).prod())
        if verbose:
            s = "%16s | %-10s | %-10s | %-10s" % ("iter of %.1e" % iterations, "loss", "term1", "term2")
            print(" " * verbose_indent + s)
            print(" " * verbose_indent + "~" * len(s))
        mll_const = d_out * sum(self._ns) * np.log(2 * np.pi)
        best, save, waited = math.inf, math.inf, 0
        best_params = None
        rec = {k: [] for k in ("loss", "scale", "lengthscales", "noise", "task_kernel")}
        for i in range(iterations + 1):
            self._cache = {k: v for k, v in self._cache.items() if not k[2]}
            if loss_metric == "GCV":
                numer, denom = self._gcv_numer_denom()
                if masks is None:
                    t1, t2 = numer, denom
                else:
                    t1 = numer[(..., *masks, slice(None))]
                    t2 = denom.expand(list(self.shape_batch) + [1])[(..., *masks, slice(None))]
                loss = (t1 / t2).sum()
                metric = loss
            elif loss_metric == "MLL":
                norm, logdet = self._norm_logdet()
                if masks is None:
                    t1 = norm.sum()
                    t2 = d_out / torch.tensor(logdet.shape).prod() * logdet.sum()
                else:
                    t1 = norm[(..., *masks, 0)].sum()
                    t2 = logdet.expand(list(self.shape_batch) + [1])[(..., *masks, 0)].sum()
                loss = 0.5 * (t1 + t2 + mll_const)
                metric = -loss
            else:
                coeffs = self.coeffs
                inv_diag = self._inv_diag()
                t1 = t2 = torch.nan * torch.ones(1)
                sq = ((coeffs / inv_diag) ** 2 * cv_weights).sum(-1, keepdim=True)
                loss = sq.sum() if masks is None else sq[(..., *masks, 0)].sum()
                metric = loss
            lv = loss.item()
            if lv < best:
                best = lv
                best_params = {k: p.data.clone() for k, p in self.named_parameters()}
            if (save - lv) > logtol:
                waited = 0
                save = best
            else:
                waited += 1
            brk = i == iterations or waited == stop_crit_wait_iterations
            if h_loss:
                rec["loss"].append(metric.item())
            if h_scale:
                rec["scale"].append(self.scale.detach().cpu())
            if h_ls:
                rec["lengthscales"].append(self.lengthscales.detach().cpu())
            if h_noise:
                rec["noise"].append(self.noise.detach().cpu())
            if h_tk:
                rec["task_kernel"].append(self.gram_matrix_tasks.detach().cpu())
            if verbose and (i % verbose == 0 or brk):
                print(" " * verbose_indent + "%16.2e | %-10.2e | %-10.2e | %-10.2e" % (
                    i, lv, t1.item() if t1.numel() == 1 else torch.nan, t2.item() if t2.numel() == 1 else torch.nan))
            if brk:
                break
            loss.backward()
            optimizer.step()
            optimizer.zero_grad()
        for k, v in best_params.items():
            setattr(self, k, torch.nn.Parameter(v, requires_grad=getattr(self, k).requires_grad))
        self._cache = {k: v for k, v in self._cache.items() if not k[2]}
        self._snap = None
        data = {"iterations": i}
        if h_loss:
            data["loss_hist"] = torch.tensor(rec["loss"])
        for k, on in (("scale", h_scale), ("lengthscales", h_ls), ("noise", h_noise), ("task_kernel", h_tk)):
            if on:
                data[k + "_hist"] = torch.stack(rec[k])
        return data

    # ------------------------------------------------------------------ predictions
    def _kmat_rows(self, x, tasks, ns):
        """[*, T', N, sum n]: Kt[t, l] K_{t,l}(x, xb_l) over the tasks l (abstract_gp.py:375,408)."""
        Kt = self.gram_matrix_tasks
        rows = []
        for t in tasks:
            blocks = []
            for l in range(self.num_tasks):
                kb = self._kmat_block(x, self.get_xb(l, ns[l]), t, l)
                blocks.append(Kt[..., t, l, None, None] * kb)
            bshape = torch.broadcast_shapes(*[b.shape[:-2] for b in blocks])
            rows.append(torch.cat([b.expand(bshape + b.shape[-2:]) for b in blocks], -1)[..., None, :, :])
        bshape = torch.broadcast_shapes(*[r.shape[:-3] for r in rows])
        return torch.cat([r.expand(bshape + r.shape[-3:]) for r in rows], -3)

    def post_mean(self, x, task=None, eval=True):
        """abstract_gp.py:352-380."""
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            coeffs = self.coeffs
            assert x.ndim == 2 and x.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
            inttask, tasks = self._task_list(task)
            x = x.to(self.device)
            kmat = self._kmat_rows(x, tasks, self._ns)
            pmean = torch.einsum("...i,...i->...", kmat, coeffs[..., None, None, :])
        return pmean[..., 0, :] if inttask else pmean

    def _check_n(self, n, msg):
        if n is None:
            return list(self._ns)
        nt = _to_n_tensor(n)
        assert ((nt & (nt - 1)) == 0).all() and nt.numel() == self.num_tasks and \
            all(int(v) >= c for v, c in zip(nt.tolist(), self._ns)), msg
        return [int(v) for v in nt.tolist()]

    def post_var(self, x, task=None, n=None, eval=True):
        """abstract_fast_gp.py:41-46 + abstract_gp.py:381-416."""
        ns = self._check_n(n, "require n are all power of two greater than or equal to self.n")
        assert x.ndim == 2 and x.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            inttask, tasks = self._task_list(task)
            x = x.to(self.device)
            Kt = self.gram_matrix_tasks
            knew = [Kt[..., t, t, None, None] * self._kmat_block(x, x, t, t, zip_pairs=True)[..., None, :]
                    for t in tasks]
            bs = torch.broadcast_shapes(*[k.shape[:-2] for k in knew])
            kmat_new = torch.cat([k.expand(bs + k.shape[-2:]) for k in knew], -2)
            kmat = self._kmat_rows(x, tasks, ns)
            nb = kmat.ndim - 3
            kperm = kmat.permute([nb, nb + 1] + list(range(nb)) + [kmat.ndim - 1])
            tperm = self.gram_matrix_solve(kperm, ns)
            t = tperm.permute(list(range(2, 2 + nb)) + [0, 1, tperm.ndim - 1])
            diag = kmat_new - (t * kmat).sum(-1)
            diag = torch.where(diag < 0, torch.zeros_like(diag), diag)
        return diag[..., 0, :] if inttask else diag

    def post_cov(self, x0, x1, task0=None, task1=None, n=None, eval=True):
        """abstract_fast_gp.py:47-52 + abstract_gp.py:417-474."""
        ns = self._check_n(n, "require n are all power of two")
        assert x0.ndim == 2 and x0.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
        assert x1.ndim == 2 and x1.size(1) == self.d, "z must a torch.Tensor with shape (-1,d)"
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            i0, t0 = self._task_list(task0)
            i1, t1 = self._task_list(task1)
            x0 = x0.to(self.device)
            x1 = x1.to(self.device)
            equal = torch.equal(x0, x1) and t0 == t1
            Kt = self.gram_matrix_tasks
            rows = []
            for a in t0:
                cols = [Kt[..., a, b, None, None] * self._kmat_block(x0, x1, a, b) for b in t1]
                bs = torch.broadcast_shapes(*[c.shape[:-2] for c in cols])
                rows.append(torch.stack([c.expand(bs + c.shape[-2:]) for c in cols], -3))
            bs = torch.broadcast_shapes(*[r.shape[:-3] for r in rows])
            kmat_new = torch.stack([r.expand(bs + r.shape[-3:]) for r in rows], -4)
            k1 = self._kmat_rows(x0, t0, ns)
            k2 = k1 if equal else self._kmat_rows(x1, t1, ns)
            nb = k2.ndim - 3
            k2p = k2.permute([nb, nb + 1] + list(range(nb)) + [k2.ndim - 1])
            tp = self.gram_matrix_solve(k2p, ns)
            t = tp.permute(list(range(2, 2 + nb)) + [0, 1, tp.ndim - 1])
            kmat = kmat_new - (k1[..., :, None, :, None, :] * t[..., None, :, None, :, :]).sum(-1)
            if equal:
                tv = torch.arange(kmat.size(-4), device=self.device)
                nv = torch.arange(x0.size(0), device=self.device)
                tm, nm = torch.meshgrid(tv, nv, indexing="ij")
                ti, ni = tm.ravel(), nm.ravel()
                dg = kmat[..., ti, ti, ni, ni]
                kmat[..., ti, ti, ni, ni] = torch.where(dg < 0, torch.zeros_like(dg), dg)
        if i0 and i1:
            return kmat[..., 0, 0, :, :]
        if i0:
            return kmat[..., 0, :, :, :]
        if i1:
            return kmat[..., :, 0, :, :]
        return kmat

    def post_cubature_mean(self, task=None, eval=True):
        """abstract_fast_gp.py:65-81."""
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            Kt = self.gram_matrix_tasks
            coeffs = self.coeffs
            inttask, tasks = self._task_list(task)
            tt = torch.tensor(tasks, device=self.device)
            cs = coeffs.split(self._ns, -1)
            sc = [(self.scale * cs[l])[..., None, :] * Kt[..., tt, l, None] for l in range(self.num_tasks)]
            bs = torch.broadcast_shapes(*[s.shape[:-1] for s in sc])
            pcmean = torch.cat([s.expand(bs + s.shape[-1:]) for s in sc], -1).sum(-1)
        return pcmean[..., 0] if inttask else pcmean

    def _inv_cut(self, ns):
        """inv[..., mvec, :, :][..., :, mvec, :][..., 0] (abstract_fast_gp.py:91,101): the inverse at the
        first row of every sorted task, frequency class 0 -> (task_order, [*G, T', T'])."""
        if self._gradmode():
            lo, A, _ = self._dense_inverse(ns)
            mv = torch.tensor(lo.rs, device=self.device)
            return lo, A[..., mv, :, :][..., :, mv, :][..., 0]
        lo, fac, _, G, gshape = self._factor(ns)
        Z = self._selinv(ns)
        T = lo.T
        cut = torch.zeros((G, T, T), dtype=torch.complex128, device=self.device)
        for (k, l) in lo.pairs:
            v = Z[:, lo.off[k, l]]
            cut[:, k, l] = v
            if k != l:
                cut[:, l, k] = v.conj()
        return lo, cut.reshape(tuple(gshape) + (T, T))

    def post_cubature_var(self, task=None, n=None, eval=True):
        """abstract_fast_gp.py:82-109."""
        ns = self._check_n(n, "require n are all power of two greater than or equal to self.n")
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            Kt = self.gram_matrix_tasks
            lo, cut = self._inv_cut(ns)
            to = torch.tensor(lo.active, device=self.device)
            nord = torch.tensor(lo.nsrt, dtype=torch.float64, device=self.device)
            nsq = torch.sqrt(nord[:, None] * nord[None, :])
            inttask, tasks = self._task_list(task)
            tt = torch.tensor(tasks, device=self.device)
            left = Kt[..., tt, :][..., :, to].to(torch.complex128)
            right = Kt[..., to, :][..., :, tt].to(torch.complex128)
            term = torch.einsum("...ij,...jk,...ki->...i", left, nsq * cut, right).real
            pcvar = self.scale * Kt[..., tt, tt] - self.scale ** 2 * term
            pcvar = torch.where(pcvar < 0, torch.zeros_like(pcvar), pcvar)
        return pcvar[..., 0] if inttask else pcvar

    def post_cubature_cov(self, task0=None, task1=None, n=None, eval=True):
        """abstract_fast_gp.py:110-154."""
        ns = self._check_n(n, "require n are all power of two greater than or equal to self.n")
        with (torch.no_grad() if eval else torch.enable_grad() if torch.is_grad_enabled() else torch.no_grad()):
            Kt = self.gram_matrix_tasks
            lo, cut = self._inv_cut(ns)
            to = torch.tensor(lo.active, device=self.device)
            nord = torch.tensor(lo.nsrt, dtype=torch.float64, device=self.device)
            nsq = torch.sqrt(nord[:, None] * nord[None, :])
            i0, t0 = self._task_list(task0)
            i1, t1 = self._task_list(task1)
            a = torch.tensor(t0, device=self.device)
            b = torch.tensor(t1, device=self.device)
            left = Kt[..., a, :][..., :, to].to(torch.complex128)
            right = Kt[..., to, :][..., :, b].to(torch.complex128)
            term = torch.einsum("...ij,...jk,...kl->...il", left, nsq * cut, right).real
            pccov = self.scale[..., None] * Kt[..., a, :][..., :, b] - self.scale[..., None] ** 2 * term
            if t0 == t1:
                tv = torch.arange(pccov.size(-1), device=self.device)
                dg = pccov[..., tv, tv]
                pccov[..., tv, tv] = torch.where(dg < 0, torch.zeros_like(dg), dg)
        if i0 and i1:
            return pccov[..., 0, 0]
        if i0:
            return pccov[..., 0, :]
        if i1:
            return pccov[..., :, 0]
        return pccov


_CLASSES = {}


def multitask_class(family_cls):
    """MultiTask<Family>: the family's transforms / point conversion over the multitask machinery
    (one class per family, created once)."""
    if family_cls not in _CLASSES:
        name = "MultiTask" + family_cls.__name__
        cls = type(name, (family_cls, MultiTaskFastGP),
                   {"__module__": __name__, "__qualname__": name, "__doc__": MultiTaskFastGP.__doc__})
        _CLASSES[family_cls] = cls
        globals()[name] = cls      # a module attribute, so pickle / torch.save find the class by name
    return _CLASSES[family_cls]


def _bind_family_classes():
    from .fast_gp import FastGPDigitalNetB2, FastGPLattice
    for fam in (FastGPLattice, FastGPDigitalNetB2):
        multitask_class(fam)


_bind_family_classes()


MT_SPECTRA_CAP = 4 << 30      # bytes of pair spectra the device-resident multitask fits may hold


class MtGeneralEngine(object):
    """Device-resident MLL fit of a general multitask / derivative-informed GP (include/fgp_hip.h ABI 14,
    fgp_mt_fit_run): the FusedMLL interface _fit_fused drives (run / loss_hist / raw_hist / split_raw), plus
    the task-kernel parameters (split_task / task_kernel_rows).

    raw = [raw_scale, raw_lengthscales (1 or d), raw_noise, raw_factor_task_kernel (T x r), raw_noise_task_kernel
    (T)]; one loss over the data batch (norm summed over B vectors, logdet weighted d_out / numel(logdet) = B,
    abstract_gp.py:252-260), gradients in closed form through the structured factor."""

    def __init__(self, gp, lr, max_iters):
        self.gp = gp
        self.device = dev = gp.device
        lo = _Layout(gp._ns)
        self.lo = lo
        spec, offs = gp._pair_spectra(lo)
        self.spec = spec
        T, d = gp.num_tasks, gp.d
        Y = lo.pack([gp.get_ytilde(l).to(torch.complex128) for l in range(T)])
        B = int(np.prod(tuple(Y.shape[:-1]))) if Y.dim() > 1 else 1
        self.y = Y.reshape(B, -1).resolve_conj().contiguous()
        # parameter batches (ABI 16): every output its own problem (G = d_out, one data vector each), its
        # parameters the rows of _mt_param_rows
        pr = gp._mt_param_rows()
        G = 1 if pr is None else B
        if G > 1:
            B = 1
            self.rows = torch.from_numpy(np.ascontiguousarray(pr[0])).to(dev)
            nrows = pr[1]
        else:
            self.rows = None
            nrows = [1] * 5
        self.G, self.B = G, B
        dl = int(gp.raw_lengthscales.shape[-1])
        r = int(gp.raw_factor_task_kernel.shape[-1])
        self.sizes = tuple(n * w for n, w in zip(nrows, gp._mt_row_widths()))
        self.raw = torch.cat([gp.raw_scale.detach().reshape(-1), gp.raw_lengthscales.detach().reshape(-1),
                              gp.raw_noise.detach().reshape(-1), gp.raw_factor_task_kernel.detach().reshape(-1),
                              gp.raw_noise_task_kernel.detach().reshape(-1)]).to(dev, torch.float64).contiguous()
        self.n_params = int(self.raw.numel())
        self.prev = torch.zeros(self.n_params, dtype=torch.float64, device=dev)
        self.step = torch.full((self.n_params,), float(lr), dtype=torch.float64, device=dev)
        self.grad = torch.zeros(self.n_params, dtype=torch.float64, device=dev)
        d_out = int(torch.tensor(tuple(gp.shape_batch)).prod()) if len(gp.shape_batch) else 1
        desc = N.MtFitDesc()
        desc.family, desc.d, desc.B = int(gp._FAMILY), int(d), B
        desc.G = G
        desc.rows = self.rows.data_ptr() if self.rows is not None else None
        for q in range(5):
            desc.nrows[q] = int(nrows[q])
        desc.layout = lo.lay
        for k, a in enumerate(lo.active):
            desc.task[k] = int(a)
        desc.T_all, desc.rank, desc.dl = int(T), r, int(dl)
        desc.spectra = self.spec.data_ptr()
        for p, o in enumerate(offs):
            desc.spec_off[p] = int(o)
        desc.y = self.y.data_ptr()
        desc.raw = self.raw.data_ptr()
        desc.vtask_exp = int(gp.tf_noise_task_kernel is _exp)
        desc.rg_scale, desc.rg_ls, desc.rg_noise = (int(gp.raw_scale.requires_grad), int(gp.raw_lengthscales.requires_grad),
                                                    int(gp.raw_noise.requires_grad))
        desc.rg_factor, desc.rg_vtask = int(gp.raw_factor_task_kernel.requires_grad), int(gp.raw_noise_task_kernel.requires_grad)
        desc.rprop_prev, desc.rprop_step, desc.grad_out = self.prev.data_ptr(), self.step.data_ptr(), self.grad.data_ptr()
        # logdet weight d_out / numel(logdet) (abstract_gp.py:256): one problem's logdet stands for the d_out outputs
        # sharing it; with a parameter batch every output is its own problem (weight 1: a parameter row shared by k
        # outputs has its logdet counted k times, as the reference's broadcast replicates it)
        w = 1.0 if G > 1 else float(d_out)
        desc.grad_norm = 0.5
        desc.grad_logdet = 0.5 * w
        desc.logdet_weight = w
        desc.mll_const = float(mll_constant(d_out, sum(gp._ns)))
        # adaptive nugget (util.py:286-290): sorted task k's trace coefficients sqrt(n_k) sum_i Phi^{kk}_S[i] and the
        # sorted position of task 0 (as _lams_blocks)
        self.nug = None
        if gp.adaptive_nugget:
            NS = 1 << d
            rows_c = []
            for k in range(lo.T):
                p = k * lo.T - k * (k - 1) // 2
                nk = lo.nsrt[k]
                blk = self.spec[offs[p]:offs[p] + NS * nk].reshape(NS, nk)
                rows_c.append(blk.sum(-1) * math.sqrt(nk))
            self.nug = torch.stack(rows_c).to(torch.complex128).contiguous()
            desc.nugget_coef = self.nug.data_ptr()
            desc.nugget_ref = lo.active.index(0) if 0 in lo.active else 0
        desc.eta_minus, desc.eta_plus = RPROP_ETAS
        desc.step_min, desc.step_max = RPROP_STEPS
        wb = ctypes.c_int64(0)
        N.call("fgp_mt_fit_work", desc, ctypes.byref(wb))
        self.work = torch.empty((max(1, wb.value),), dtype=torch.uint8, device=dev)
        desc.work = self.work.data_ptr()
        npar = ctypes.c_int(0)
        N.call("fgp_mt_fit_nparams", desc, ctypes.byref(npar))
        assert npar.value == self.n_params
        self.desc = desc
        self.max_iters = 0
        self.loss_hist = None
        self.raw_hist = None
        self.ensure_history(max_iters)

    def ensure_history(self, iters):
        if iters <= self.max_iters:
            return
        new_max = max(iters, 2 * self.max_iters, 16)
        lh = torch.zeros((new_max, 1, 3), dtype=torch.float64, device=self.device)
        rh = torch.zeros((new_max, self.n_params), dtype=torch.float64, device=self.device)
        if self.loss_hist is not None:
            lh[:self.max_iters] = self.loss_hist
            rh[:self.max_iters] = self.raw_hist
        self.loss_hist, self.raw_hist, self.max_iters = lh, rh, new_max
        self.desc.loss_hist, self.desc.raw_hist = lh.data_ptr(), rh.data_ptr()

    def run(self, iter0, iters, final_no_update=False):
        self.ensure_history(iter0 + iters)
        N.call("fgp_mt_fit_run", self.desc, int(iter0), int(iters), int(bool(final_no_update)),
               N.stream_ptr(self.device))

    def _cut(self, raw_vec, i):
        o = sum(self.sizes[:i])
        return raw_vec[..., o:o + self.sizes[i]]

    def split_raw(self, raw_vec):
        return self._cut(raw_vec, 0), self._cut(raw_vec, 1), self._cut(raw_vec, 2)

    def split_task(self, raw_vec):
        return self._cut(raw_vec, 3), self._cut(raw_vec, 4)

    def task_kernel_rows(self, raw_rows):
        """K_task = F F^T + diag(v) of every history row (util.py:157-162)."""
        gp = self.gp
        f, v = self.split_task(raw_rows)
        F = gp.tf_factor_task_kernel(f.reshape((-1,) + tuple(gp.raw_factor_task_kernel.shape)))
        vv = gp.tf_noise_task_kernel(v.reshape((-1,) + tuple(gp.raw_noise_task_kernel.shape)))
        FF, V = torch.einsum("...il,...kl->...ik", F, F), torch.diag_embed(vv)
        # batch dims broadcast right-aligned after the leading history dim
        nb = max(FF.dim(), V.dim())
        FF = FF.reshape(FF.shape[:1] + (1,) * (nb - FF.dim()) + FF.shape[1:])
        V = V.reshape(V.shape[:1] + (1,) * (nb - V.dim()) + V.shape[1:])
        return FF + V
