"""Drop-in FastGPLattice / FastGPDigitalNetB2 on MI355X.

Host-side mirror of the reference's Python interface (alegresor/FastGaussianProcesses, fastgps
0.0.4.1a): same constructor keywords (fast_gp_lattice.py:125-158, fast_gp_digital_net_b2.py:120-153),
same methods and return shapes (abstract_gp.py, abstract_fast_gp.py), same assertion messages for
misuse.  Every numerical hot spot runs in the HIP library (include/fgp_hip.h):

  ft / ift                  -> fgp_fftbr / fgp_ifftbr / fgp_fwht (stable, differentiable)
  k1 parts                  -> fgp_lattice_parts / fgp_net_parts
  fit (MLL, default Rprop)  -> fgp_fit_run: fused forward / adjoint / Rprop on device, histories read
                               back in chunks to apply the reference's early-stopping rule exactly
  post_mean                 -> fgp_post_mean (matrix-free cross-kernel contraction)
  post_var / post_cov       -> fgp_kernel_rows + the transform solve

This module holds single-task GPs (num_tasks=None or 1) without derivative information
(beta = kappa = 0); multitask (num_tasks > 1) and derivative-informed GPs are built by the same
constructors and run multitask.py.  Hyper-parameter fits other than (MLL, default optimizer, no
masks, default log/exp transforms) run a generic path: torch autograd through the HIP transforms and
torch device ops, with the caller's torch optimizer.
"""
import math
import os

import numpy as np
import scipy.stats
import torch

from . import _native
from . import ops
from . import seqs as _seqs
from .fit_engine import (SPEC_MAX_D, FusedMLL, LatticePartsGen, cached_engine, mll_constant, spec_basis, spec_basis_gen,
                         spec_inv_eig, spec_k, spec_post_var, spectral_wanted)


def _log(x):
    return torch.log(x)


def _exp(x):
    return torch.exp(x)


def _identity(x):
    return x


_DEFAULT_TFS = (_log, _exp)
_IDENTITY_TFS = (_identity, _identity)     # module-level functions: a GP pickles (torch.save) whole
SPEC_POST_VAR_MAX_N = 4096            # test points per fgp_spec_post_var call (include/fgp_hip.h)
SPEC_POST_VAR_WORK = 1 << 30          # bytes of row products + row spectra per slice of test points


def _as_size(s):
    if s is None or isinstance(s, torch.Size):
        return s
    return torch.Size(s)


class _Hyper(object):
    """Resolves one hyper-parameter's shape exactly as AbstractGP.__init__ (abstract_gp.py:78-139)."""

    @staticmethod
    def make(value, shape, shape_batch, last_ok, name, positive, device, core=1):
        assert np.isscalar(value) or isinstance(value, torch.Tensor), "%s must be a scalar or torch.Tensor" % name
        if isinstance(value, torch.Tensor):
            shape = value.shape
        shape = _as_size(shape)
        assert isinstance(shape, torch.Size) and last_ok(shape[-1])
        if len(shape) > core:   # leading dims must be a suffix of shape_batch
            assert shape[:-core] == shape_batch[-(len(shape) - core):]
        if np.isscalar(value):
            value = value * torch.ones(shape, device=device)
        value = value.to(device=device, dtype=torch.float64)
        if positive == "pos":
            assert (value > 0).all(), "%s must be positive" % name
        elif positive == "nonneg":
            assert (value >= 0).all(), "%s must be positive" % name
        return value


def _trivial_derivatives(derivatives, derivatives_coeffs):
    """derivatives / derivatives_coeffs that leave a one-task GP's kernel unchanged: ONE all-zero derivative
    row (beta = 0) with coefficient 1 -- e.g. the probnum25 paper's `derivatives=[torch.zeros((1, d))]`
    ($f$ columns of benchmarks_accuracy_time.tex).  None counts as trivial."""
    if derivatives is not None:
        v = derivatives[0] if isinstance(derivatives, (list, tuple)) and len(derivatives) == 1 else derivatives
        if not isinstance(v, torch.Tensor):
            return False
        v = v.reshape(-1, v.shape[-1]) if v.ndim else v
        if v.ndim != 2 or v.shape[0] != 1 or bool((v != 0).any()):
            return False
    if derivatives_coeffs is not None:
        c = derivatives_coeffs[0] if isinstance(derivatives_coeffs, (list, tuple)) and len(derivatives_coeffs) == 1 \
            else derivatives_coeffs
        if not isinstance(c, torch.Tensor) or c.numel() != 1 or float(c.reshape(-1)[0]) != 1.0:
            return False
    return True


def _wants_multitask(cls, args, kwargs):
    """num_tasks > 1, or non-trivial derivative information, in a family constructor's arguments.  One task
    with trivial derivatives (_trivial_derivatives) is the single-task GP: the reference's general path gives
    it the same loss and predictions (rank-1 task factor 1, task noise 0: gram_matrix_tasks == 1,
    abstract_gp.py:58-72), so it takes the single-task fused kernels."""
    import inspect
    bound = inspect.signature(cls.__init__).bind_partial(None, *args, **kwargs).arguments
    nt = bound.get("num_tasks")
    return (nt is not None and nt != 1) or not _trivial_derivatives(bound.get("derivatives"),
                                                                    bound.get("derivatives_coeffs")) \
        or _nonunit_task_kernel(bound)


def _nonunit_task_kernel(bound):
    """A single-task GP whose task kernel is not the constant 1: num_tasks = 1 keeps rank 0 (no factor), so
    gram_matrix_tasks = noise_task_kernel (abstract_gp.py:116-139); a value != 1, a factor of positive rank
    or a learned task kernel scales every eigenvalue (ev = (sqrt(n) lambda + noise) Kt, util.py:285-298) and
    every kernel row (abstract_gp.py:375) -- the multitask class (T = 1) carries that."""
    learned = bool(bound.get("requires_grad_noise_task_kernel")) or bool(bound.get("requires_grad_factor_task_kernel"))
    if bound.get("derivatives") is not None or bound.get("derivatives_coeffs") is not None:
        # derivative information: rank-1 factor, task noise 0 (abstract_gp.py:58-62) -> Kt = factor^2
        f = bound.get("factor_task_kernel", 1.0)
        f2 = (f.reshape(-1) ** 2).sum() if isinstance(f, torch.Tensor) else f * f
        return learned or not bool(f2 == 1)
    v = bound.get("noise_task_kernel", 1.0)
    unit = bool((v == 1).all()) if isinstance(v, torch.Tensor) else (v == 1)
    r, sf = bound.get("rank_factor_task_kernel"), bound.get("shape_factor_task_kernel")
    f = bound.get("factor_task_kernel")
    factor = (r not in (None, 0)) or (sf is not None and tuple(sf)[-1] != 0) or \
        (isinstance(f, torch.Tensor) and f.shape[-1] != 0)
    return (not unit) or factor or learned


class AbstractFastGP(torch.nn.Module):
    """Shared machinery of FastGPLattice / FastGPDigitalNetB2 (single task, beta=kappa=0).

    Constructing FastGPLattice / FastGPDigitalNetB2 with num_tasks > 1 or with derivatives /
    derivatives_coeffs returns the family's multitask class instead (multitask.py)."""

    _FAMILY = None
    _XBDTYPE = None
    _FTOUTDTYPE = None
    _MULTITASK = False
    # host-side attributes the fit / ingest path reassigns on every call (never Parameters, buffers or sub-modules)
    _PLAIN_ATTRS = frozenset(("_cache", "_snap", "_nh", "_y", "_yt_state", "_n_t", "_m_t", "_iters_for_log",
                              "_pgen_memo", "_task_unit_memo", "_pts_T", "_pts_n", "_x", "_xb"))

    def __new__(cls, *args, **kwargs):
        if not cls._MULTITASK and cls._FAMILY is not None and _wants_multitask(cls, args, kwargs):
            from .multitask import multitask_class
            cls = multitask_class(cls)
        return super().__new__(cls)

    def __init__(self, seqs, num_tasks, seed_for_seq, alpha, scale, lengthscales, noise, factor_task_kernel,
                 rank_factor_task_kernel, noise_task_kernel, device, tfs_scale, tfs_lengthscales, tfs_noise,
                 tfs_factor_task_kernel, tfs_noise_task_kernel, requires_grad_scale, requires_grad_lengthscales,
                 requires_grad_noise, requires_grad_factor_task_kernel, requires_grad_noise_task_kernel, shape_batch,
                 shape_scale, shape_lengthscales, shape_noise, shape_factor_task_kernel, shape_noise_task_kernel,
                 derivatives, derivatives_coeffs, compile_fts, compile_fts_kwargs, adaptive_nugget,
                 data_dtype=torch.float64):
        super().__init__()
        assert torch.get_default_dtype() == torch.float64, \
            "fast transforms do not work without torch.float64 precision"
        if num_tasks is None:
            self.solo_task, self.default_task, num_tasks = True, 0, 1
        else:
            assert isinstance(num_tasks, int) and num_tasks > 0
            self.solo_task, self.default_task = False, torch.arange(num_tasks)
        if num_tasks != 1 or not _trivial_derivatives(derivatives, derivatives_coeffs):
            raise AssertionError("multitask / derivative-informed GPs are built through FastGPLattice / "
                                 "FastGPDigitalNetB2 (multitask.py)")
        if derivatives is not None or derivatives_coeffs is not None:
            # the reference's derivative settings (abstract_gp.py:58-62): rank-1 task factor, task noise 0
            rank_factor_task_kernel = 1
            tfs_noise_task_kernel = _IDENTITY_TFS
            noise_task_kernel = 0.
        self.num_tasks = 1
        # Extension (not in the reference, which is fp64-only, abstract_gp.py:46): data_dtype=float32
        # stores the observations in fp32 and forms the MLL's data term from a complex64 ytilde
        # (fgp_fftbr_c64, Y = sum |ytilde|^2 accumulated in fp64) -- the mixed-precision path of
        # BASELINE config C5.  Eigenvalues, the MLL / gradient / Rprop loop, the coefficients
        # (fp64 transform of the fp32 observations), post_mean and post_var stay fp64.
        assert data_dtype in (torch.float64, torch.float32), "data_dtype must be torch.float64 or torch.float32"
        self.data_dtype = data_dtype
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("fastgaussianprocesses_amd runs on a HIP device (device='cuda'); got %s" % device)
        self.seq = self._resolve_seq(seqs, seed_for_seq)
        self.seqs = np.array([self.seq], dtype=object)
        self.d = int(self.seq.d)
        # the (trivial) derivative specification (abstract_gp.py:63-72)
        self.derivatives = [torch.zeros((1, self.d), dtype=torch.int64, device=self.device)]
        self.derivatives_coeffs = [torch.ones(1, device=self.device)]
        # shape_batch / hyper-parameters (abstract_gp.py:73-139)
        shape_batch = _as_size(shape_batch)
        assert isinstance(shape_batch, torch.Size)
        self.shape_batch = shape_batch
        self.ndim_batch = len(shape_batch)
        d = self.d
        dev = self.device
        scale = _Hyper.make(scale, shape_scale, shape_batch, lambda v: v == 1, "scale", "pos", dev)
        if shape_lengthscales is None and not isinstance(lengthscales, torch.Tensor):
            shape_lengthscales = torch.Size([d])
        lengthscales = _Hyper.make(lengthscales, shape_lengthscales, shape_batch, lambda v: v in (1, d),
                                   "lengthscales", "pos", dev)
        noise = _Hyper.make(noise, shape_noise, shape_batch, lambda v: v == 1, "noise", "pos", dev)
        # the default task kernel (no factor columns, task noise 1 through the default transforms) is exactly 1:
        # known here, so the first fit need not check it on the device (_task_unit)
        unit_task = (shape_factor_task_kernel is None and not isinstance(factor_task_kernel, torch.Tensor)
                     and not rank_factor_task_kernel and shape_noise_task_kernel is None
                     and not isinstance(noise_task_kernel, torch.Tensor) and float(noise_task_kernel) == 1.0
                     and tfs_noise_task_kernel is _DEFAULT_TFS)
        if shape_factor_task_kernel is None and not isinstance(factor_task_kernel, torch.Tensor):
            if rank_factor_task_kernel is None:
                rank_factor_task_kernel = 0
            shape_factor_task_kernel = torch.Size([1, rank_factor_task_kernel])
        factor_task_kernel = _Hyper.make(factor_task_kernel, shape_factor_task_kernel, shape_batch,
                                         lambda v: 0 <= v <= 1, "factor_task_kernel", None, dev, core=2)
        if shape_noise_task_kernel is None and not isinstance(noise_task_kernel, torch.Tensor):
            shape_noise_task_kernel = torch.Size([1])
        noise_task_kernel = _Hyper.make(noise_task_kernel, shape_noise_task_kernel, shape_batch, lambda v: v == 1,
                                        "noise_task_kernel", "nonneg", dev)
        for tfs in (tfs_scale, tfs_lengthscales, tfs_noise, tfs_factor_task_kernel, tfs_noise_task_kernel):
            assert len(tfs) == 2 and callable(tfs[0]) and callable(tfs[1]), \
                "tfs should be a tuple of two callables, the transform and inverse transform"
        self._tfs = dict(scale=tfs_scale, lengthscales=tfs_lengthscales, noise=tfs_noise)
        self.tf_scale, self.tf_lengthscales, self.tf_noise = tfs_scale[1], tfs_lengthscales[1], tfs_noise[1]
        self.tf_factor_task_kernel, self.tf_noise_task_kernel = tfs_factor_task_kernel[1], tfs_noise_task_kernel[1]
        self.raw_scale = torch.nn.Parameter(tfs_scale[0](scale), requires_grad=requires_grad_scale)
        self.raw_lengthscales = torch.nn.Parameter(tfs_lengthscales[0](lengthscales),
                                                   requires_grad=requires_grad_lengthscales)
        self.raw_noise = torch.nn.Parameter(tfs_noise[0](noise), requires_grad=requires_grad_noise)
        self.raw_factor_task_kernel = torch.nn.Parameter(tfs_factor_task_kernel[0](factor_task_kernel),
                                                         requires_grad=bool(requires_grad_factor_task_kernel))
        self.raw_noise_task_kernel = torch.nn.Parameter(tfs_noise_task_kernel[0](noise_task_kernel),
                                                        requires_grad=bool(requires_grad_noise_task_kernel))
        if unit_task:
            self._task_unit_memo = (self._task_unit_key(), True)
        self.adaptive_nugget = adaptive_nugget
        self.compile_fts, self.compile_fts_kwargs = compile_fts, compile_fts_kwargs   # accepted; HIP kernels are native
        # alpha (abstract_fast_gp.py:21-24)
        assert (np.isscalar(alpha) and alpha % 1 == 0) or (isinstance(alpha, torch.Tensor) and alpha.shape == (self.d,)), \
            "alpha should be an int or a torch.Tensor of length d"
        if np.isscalar(alpha):
            alpha = int(alpha) * torch.ones(self.d, dtype=torch.int64, device=dev)
        self.alpha = alpha
        self._alphas = [int(a) for a in alpha.tolist()]
        # data
        self.n = torch.zeros(1, dtype=torch.int64, device=dev)
        self.m = -torch.ones(1, dtype=torch.int64, device=dev)
        self._nh = 0           # host mirror of self.n[0] (no device syncs on the hot path)
        self._y = [torch.empty(0, device=dev)]
        self._pts_n = 0
        self._x = torch.empty((0, self.d), device=dev)
        self._xb = torch.empty((0, self.d), dtype=self._XBDTYPE, device=dev)
        self._parts = {}       # n -> [d, n] first-column parts
        self._cache = {}       # derived quantities keyed by (name, n) + parameter snapshot
        self._snap = None

    def __setattr__(self, name, value):
        """nn.Module.__setattr__ costs ~3 us a call (its Parameter / buffer / sub-module bookkeeping) and a fit + ingest
        makes ~20 of them: the plain host attributes above are set directly, and a Parameter replacing an existing one
        (AbstractGP.fit's best-iterate restore, abstract_gp.py:295-296) goes straight into _parameters, which is where
        register_parameter would put it (global parameter-registration hooks are not run for such replacements)."""
        if name in self._PLAIN_ATTRS:
            object.__setattr__(self, name, value)
        elif type(value) is torch.nn.Parameter and name in self.__dict__["_parameters"]:
            self.__dict__["_parameters"][name] = value
        else:
            super().__setattr__(name, value)

    @property
    def n(self):
        """Samples so far ([1] int64 on the device, the reference's gp.n): formed when first read after add_y_next
        (the fit path reads the host mirror _nh; two device fills per ingest saved)."""
        t = self._n_t
        if t is None:
            t = self._n_t = torch.full((1,), self._nh, dtype=torch.int64, device=self.device)
        return t

    @n.setter
    def n(self, v):
        self._n_t = v

    @property
    def m(self):
        """log2 of n ([1] int64 on the device, -1 without samples), formed on first read like n."""
        t = self._m_t
        if t is None:
            t = self._m_t = torch.full((1,), self._nh.bit_length() - 1 if self._nh > 0 else -1, dtype=torch.int64,
                                       device=self.device)
        return t

    @m.setter
    def m(self, v):
        self._m_t = v

    # ------------------------------------------------------------------ construction helpers
    def _resolve_seq(self, seqs, seed_for_seq):
        if isinstance(seqs, (int, np.integer)):
            seed = np.random.SeedSequence(seed_for_seq).spawn(1)[0]
            return self._default_seq(int(seqs), seed)
        if isinstance(seqs, (list, np.ndarray)):
            seqs = list(seqs)
            assert len(seqs) == 1, "seqs should be a length num_tasks=1 list"
            seqs = seqs[0]
        self._check_seq(seqs)
        return seqs

    # ------------------------------------------------------------------ hyper-parameters
    @property
    def scale(self):
        return self.tf_scale(self.raw_scale)

    @property
    def lengthscales(self):
        return self.tf_lengthscales(self.raw_lengthscales)

    @property
    def noise(self):
        return self.tf_noise(self.raw_noise)

    @property
    def factor_task_kernel(self):
        return self.tf_factor_task_kernel(self.raw_factor_task_kernel)

    @property
    def noise_task_kernel(self):
        return self.tf_noise_task_kernel(self.raw_noise_task_kernel)

    @property
    def gram_matrix_tasks(self):
        """F F^T + diag(noise_task_kernel) (util.py:157-162)."""
        F = self.factor_task_kernel
        k = torch.einsum("...il,...kl->...ik", F, F)
        return k + self.noise_task_kernel[..., None] * torch.eye(1, device=self.device)

    @property
    def total_parameters(self):
        return sum(p.numel() for p in self.parameters())

    @property
    def total_tuneable_parameters(self):
        return sum((p.numel() if p.requires_grad else 0) for p in self.parameters())

    def get_default_optimizer(self, lr):
        return torch.optim.Rprop(self.parameters(), lr=1e-1 if lr is None else lr)

    def _param_key(self):
        # identity + version counter of every raw hyper-parameter: in-place updates (optimizer steps)
        # bump the version, reassignment changes the identity -- no device synchronisation needed
        return tuple((id(p), p._version, p.data_ptr()) for p in (
            self.raw_scale, self.raw_lengthscales, self.raw_noise, self.raw_factor_task_kernel,
            self.raw_noise_task_kernel))

    def _params_changed(self):
        key = self._param_key()
        if self._snap != key:
            self._snap = key
            return True
        return False

    def _hparams(self):
        return (self.raw_scale, self.raw_lengthscales, self.raw_noise, self.raw_factor_task_kernel,
                self.raw_noise_task_kernel)

    def _gradmode(self):
        """True when results must carry an autograd graph w.r.t. the hyper-parameters."""
        return torch.is_grad_enabled() and any(p.requires_grad for p in self._hparams())

    def _cached(self, key, fn, grad_sensitive=True):
        """Cache a derived quantity until n or the hyper-parameters change (the reference's
        _frozen_equal / FASTGP_FORCE_RECOMPILE invalidation, util.py:81-94,185-205).  Values computed
        with and without an autograd graph are cached separately; graph-free ones come from the
        fused HIP paths."""
        if self._params_changed():
            self._cache = {k: v for k, v in self._cache.items() if not k[2]}
        k = (key[0], key[1], grad_sensitive, grad_sensitive and self._gradmode())
        if k not in self._cache:
            self._cache[k] = fn()
        return self._cache[k]

    def _task_unit(self):
        """gram_matrix_tasks == 1 (a single-task GP's unit task kernel).  Checked again only when the
        task-kernel parameters change: the check synchronises with the device."""
        key = self._task_unit_key()
        hit = getattr(self, "_task_unit_memo", None)
        if hit is None or len(hit[0]) != len(key) or not all(
                a[0] is b[0] and a[1:] == b[1:] for a, b in zip(hit[0], key)):
            kt = self.gram_matrix_tasks.detach()
            hit = self._task_unit_memo = (key, bool(torch.equal(kt, torch.ones_like(kt))))
        return hit[1]

    def _task_unit_key(self):
        """The task-kernel Parameters THEMSELVES (held by the memo, so a replaced Parameter's id / address cannot
        be reused by a new one while the memo refers to it), their version counters and data pointers."""
        return tuple((p, p._version, p.data_ptr()) for p in (self.raw_factor_task_kernel, self.raw_noise_task_kernel))

    def _task_scalar(self):
        if not self._task_unit():
            raise NotImplementedError("single-task GPs with a non-unit task kernel are not supported")
        return 1.0

    # ------------------------------------------------------------------ points and data
    def _ensure_points(self, n):
        n = int(n)
        if n <= self._pts_n:
            return
        x, xb = self._sample(self._pts_n, n)
        self._x = torch.cat([self._x, x], 0)
        self._xb = x if self._XBDTYPE == torch.float64 else torch.cat([self._xb, xb], 0)
        if self._XBDTYPE == torch.float64:
            self._xb = self._x
        self._pts_n = n

    def _points_T(self, n):
        """[d, n] dimension-major copy of the first n points (cached: points only ever grow)."""
        n = int(n)
        self._ensure_points(n)
        pt = getattr(self, "_pts_T", None)
        if pt is None or pt[0] != n:
            self._pts_T = (n, self._xb[:n].T.contiguous())
        return self._pts_T[1]

    def get_x(self, task=0, n=None):
        assert task == 0
        n = self._nh if n is None else int(n)
        assert n >= 0
        self._ensure_points(n)
        return self._x[:n]

    def get_xb(self, task=0, n=None):
        assert task == 0
        n = self._nh if n is None else int(n)
        assert n >= 0
        self._ensure_points(n)
        return self._xb[:n]

    def get_x_next(self, n, task=None):
        n_og = n
        if isinstance(n, (int, np.int64)):
            n = torch.tensor([n], dtype=torch.int64)
        if isinstance(n, list):
            n = torch.tensor(n, dtype=torch.int64)
        assert isinstance(n, torch.Tensor) and torch.logical_or(n == 0, n & (n - 1) == 0).all(), \
            "maximum sequence index must be a power of 2"
        if task is None:
            task = self.default_task
        inttask = isinstance(task, int)
        ns = n.tolist()
        assert all(v >= self._nh for v in ns), \
            "maximum sequence index must be greater than the current number of samples"
        out = [self.get_x(0, v)[self._nh:v] for v in ns]
        return out[0] if inttask else out

    def add_y_next(self, y_next, task=None):
        if isinstance(y_next, torch.Tensor):
            y_next = [y_next]
        assert isinstance(y_next, list) and len(y_next) == 1
        assert all(y.shape[:-1] == self.shape_batch for y in y_next)
        y = y_next[0].to(device=self.device, dtype=self.data_dtype)
        old = int(self._y[0].size(-1))
        st = getattr(self, "_yt_state", None)
        if st is None or old == 0 or st[0] > old or old != self._nh:
            self._yt_state = None           # only an append keeps the cached prefix transform valid
        self._y[0] = torch.cat([self._y[0].to(self.data_dtype), y], -1)
        self._nh = int(self._y[0].size(-1))
        # gp.n / gp.m: device fills on first read (properties above), not host->device copies (a pageable copy blocks)
        self._n_t = self._m_t = None
        self._cache = {}
        assert self._nh == 0 or (self._nh & (self._nh - 1)) == 0, "total samples must be power of 2"

    @property
    def x(self):
        return self.get_x(0)

    @property
    def y(self):
        return self._y[0]

    # ------------------------------------------------------------------ transforms (plugin point)
    def ft(self, x):
        """Stable forward transform along the last dim (abstract_fast_gp.py:197-212), HIP kernels."""
        raise NotImplementedError

    def ift(self, x):
        raise NotImplementedError

    # ------------------------------------------------------------------ kernel pieces
    def _k1parts(self, n, out=None):
        """[d, n] first-column kernel parts (cached per n; `out` places them in a caller buffer)."""
        n = int(n)
        if n not in self._parts or (out is not None and self._parts[n].data_ptr() != out.data_ptr()):
            self._ensure_points(n)
            if out is not None and n in self._parts:
                out.copy_(self._parts[n])
            else:
                out = self._compute_parts(self._xb[:n], self._xb[0], out)
            self._parts[n] = out
        return self._parts[n]

    def _parts_gen(self, n):
        """Parts generator for the fused kernels (None: read the cached parts array)."""
        return None

    def get_k1parts(self, task0=0, task1=0, n=None):
        n = self._nint(n)
        return self._k1parts(n).T[:, None, None, :]

    def _k1(self, n, parts=None):
        """k1 = scale * prod_j(1 + l_j parts_j)  -> [*param_batch, n] (abstract_fast_gp.py:181-191)."""
        parts = self._k1parts(n) if parts is None else parts
        ls = self.lengthscales
        factors = 1 + ls[..., :, None] * parts          # [*lb, d, n]
        return self.scale * factors.prod(-2)

    def _nint(self, n):
        return self._nh if n is None else int(torch.as_tensor(n).reshape(-1)[0])

    def get_lam(self, task0=0, task1=0, n=None):
        n = self._nint(n)

        def f():
            if not self._gradmode():
                half = self._cache.get(("lam", n // 2, True, False)) if n >= 4 else None
                if half is not None:
                    # _LamCaches doubling (util.py:113-132): lam_n from the cached lam_{n/2} and ft of the
                    # first-column kernel over the new half of the points, one DIT stage
                    self._ensure_points(n)
                    parts = self._compute_parts(self._xb[n // 2:n], self._xb[0])
                    return ops.double_update(self._FAMILY, half, self.ft(self._k1(n // 2, parts)))
                if self._lam_fusable(n):
                    return self._lam_fused(n)
            return self.ft(self._k1(n))
        return self._cached(("lam", n), f)

    def _lam_fusable(self, n):
        return (n >= 16 and self.d <= 8 and self._tfs["scale"][1] is _exp and self._tfs["lengthscales"][1] is _exp
                and self._tfs["noise"][1] is _exp and self._problem_batch() is not None)

    def _lam_fused(self, n):
        """lambda = ft(k1) by fgp_nll_lam (k1 formed on the fly from the cached parts, or lambda from the
        part-product spectra on the spectral path)."""
        from .fit_engine import fused_lam
        pb, G = self._problem_batch()
        basis = self._spec_basis(n, G)
        gen = self._parts_gen(n) if basis is None else None
        parts = self._k1parts(n) if (gen is None and basis is None) else None
        lam = fused_lam(self._FAMILY, parts, self.raw_scale.detach().reshape(-1),
                        self.raw_lengthscales.detach().reshape(-1, self.raw_lengthscales.shape[-1]),
                        self.raw_noise.detach().reshape(-1), G, gen=gen, n=n, basis=basis)
        return lam.reshape(tuple(pb) + (n,))

    def _spec_basis(self, n, G=1, force=False):
        """Part-product spectra Phi_S = ft(prod_{j in S} parts_j) of the first n points (fgp_spec_basis)
        when the spectral fit path is the cheaper one for G eigen-problems (fit_engine.spectral_wanted), or
        with `force` whenever it applies (d <= 6, the spectra <= 16 GiB: the GCV / CV fits, which only it runs),
        else None.  Hyper-parameter independent; cached with the data (dropped by add_y_next)."""
        if force:
            if self.d > SPEC_MAX_D or n < 16 or (2 ** self.d) * spec_k(self._FAMILY, n) * 8 > (16 << 30):
                return None
        elif not spectral_wanted(self._FAMILY, n, self.d, G):
            return None

        def f():
            gen = self._parts_gen(n)
            if gen is not None:
                b = spec_basis_gen(gen, n, self.device)      # the parts regenerated in the transform
                if b is not None:
                    return b
            if gen is not None:
                # the regenerated parts, kept per n like the parts array (_k1parts): a function of the points only,
                # so a later add_y_next at this n (or new data at the same points) does not regenerate them
                memo = self.__dict__.setdefault("_parts_regen", {})
                hit = memo.get(n)
                if hit is None or hit[0] is not gen:
                    hit = memo[n] = (gen, ops.lattice_parts_gen(gen.z, gen.shift[0], gen.alphas, n))
                parts = hit[1]
            else:
                parts = self._k1parts(n)
            return spec_basis(self._FAMILY, parts, n)
        return self._cached(("basis", n), f, grad_sensitive=False)

    def get_ytilde(self, task=0):
        """_YtildeCache (util.py:164-183): after add_y_next doubled n, ytilde_2n comes from the cached
        ytilde_n and ft of the NEW half by one DIT stage (fgp_double_update), as the reference does,
        instead of a full-length transform."""
        n = self._nh

        def f():
            y = self._y[0]
            st = getattr(self, "_yt_state", None)
            half = self._cache.get(("ytilde_half", n, False, False)) if y.dtype == torch.float64 else None
            if half is not None:
                # the fused consumers took only the Hermitian half (_ytilde_half): the full spectrum is its mirror
                yt = ops.hermitian_full(half, n)
            elif st is not None and 1 < st[0] < n and y.dtype == torch.float64 and n % st[0] == 0:
                ns, yt = st
                while ns < n:
                    yt = ops.double_update(self._FAMILY, yt, self.ft(y[..., ns:2 * ns]))
                    ns *= 2
            else:
                yt = self.ft(y) if n > 1 else y.clone().to(self._FTOUTDTYPE)
            self._yt_state = (n, yt)
            return yt
        return self._cached(("ytilde", n), f, grad_sensitive=False)

    def _ytilde_half(self):
        """The Hermitian half (k <= n/2) of ytilde = ft(y) of real float64 / float32 lattice observations, 2^17 <= n <= 2^24
        (ops.fftbr_real_half): all that Y = sum |ytilde|^2 and the spectral coefficient solve read, at half the
        bytes written; a view of the full ytilde when that is cached already.  None when it does not apply."""
        n = self._nh
        y = self._y[0]
        if self._FAMILY != ops.LATTICE or n < 2 or not ops.half_spectrum_ok(y):
            return None
        if y.dtype == torch.float32:
            # data_dtype=float32: the fp32 rows widened exactly on load (fgp_fftbr_real_half_f32) -- Y and the
            # coefficients in fp64 from one transform; get_ytilde keeps the API's complex64 ft(y)
            return self._cached(("ytilde_half64", n), lambda: ops.fftbr_real_half(y), grad_sensitive=False)
        full = self._cache.get(("ytilde", n, False, False))
        if full is not None:
            return full[..., :n // 2 + 1]
        st = getattr(self, "_yt_state", None)
        if st is not None and 1 < st[0] < n and n % st[0] == 0:
            return None                           # the doubling update of the cached ytilde (get_ytilde) is cheaper
        return self._cached(("ytilde_half", n), lambda: ops.fftbr_real_half(y), grad_sensitive=False)

    def _ev(self, n):
        """sqrt(n) lam + noise (util.py:285,292-298, single task; adaptive nugget: util.py:286-290)."""
        lam = self.get_lam(0, 0, n)
        ev = math.sqrt(n) * lam
        if self.adaptive_nugget:
            ev = ev + self.noise * (ev.sum(-1, keepdim=True) / ev.sum(-1, keepdim=True)).abs()
        else:
            ev = ev + self.noise
        return ev * self._task_scalar()

    def get_inv_log_det(self, n=None):
        n = self._nint(n)

        def f():
            ev = self._ev(n)
            return (1 / ev)[..., None, None, :], torch.log(torch.abs(ev)).sum(-1)
        return self._cached(("invlogdet", n), f)

    def _inv(self, n):
        return self.get_inv_log_det(n)[0][..., 0, 0, :]

    def _solve(self, v, n):
        """K^-1 v = ift(A ft(v)).real (util.py:338-353)."""
        return self.ift(self.ft(v) * self._inv(n)).real

    def _coeffs_now(self):
        n = self._nh
        if self._gradmode() or n < 2:
            # data_dtype=float32: the coefficients still come from an fp64 transform (as the graph-free
            # branch below), so both modes give the same posterior mean
            y = self._y[0]
            return self._solve(y if y.dtype == torch.float64 else y.to(torch.float64), n)
        # graph-free: reuse the cached ytilde = ft(y); A * ytilde fused into the inverse transform's
        # first pass and its real part into the last (fgp_ifftbr_mul).  data_dtype=float32: the
        # coefficients still come from an fp64 transform of the (fp32) observations -- cond(K) ~ n /
        # noise makes fp32 coefficients useless for the posterior mean (measured O(1) relative error,
        # tools/diag_mixed.py of round 3, in git history), so only the MLL's Y uses the complex64 ytilde.
        rows_y = self._y[0].numel() // n
        pb = self._problem_batch() if (self._lam_fusable(n) and not self.adaptive_nugget) else None
        basis = None
        if (pb is not None and self._FAMILY == ops.LATTICE and 17 <= n.bit_length() - 1 <= 24
                and pb[1] in (1, rows_y)):
            basis = self._spec_basis(n, pb[1])
        half = self._ytilde_half() if basis is not None else None
        if half is not None:
            yt = half                     # the Hermitian half is all fgp_ifftbr_real_rf reads
        elif self.data_dtype != torch.float64:
            y = self._y[0].to(torch.float64)
            yt = ops.fftbr_raw(y, stable=True) if self._FAMILY == ops.LATTICE else ops.fwht_raw(y, stable=True)
        else:
            yt = self.get_ytilde(0)
        if basis is not None:
            # spectral path: the real A = 1/ev straight from the part-product spectra (fgp_spec_inv_eig; one
            # row shared by every output, or one per output's eigen-problem), the product fused into the
            # half-length real inverse (fgp_ifftbr_real_rf) -- no lambda, no ytilde * A array
            self._task_scalar()
            wa = spec_inv_eig(self._FAMILY, self.raw_scale.detach().reshape(-1),
                              self.raw_lengthscales.detach().reshape(-1, self.raw_lengthscales.shape[-1]),
                              self.raw_noise.detach().reshape(-1), pb[1], n, basis)
            self._cached(("inv_real", n), lambda: wa.reshape(tuple(pb[0]) + (n,)))
            return ops.ifftbr_real_rf(yt, wa, n=n)
        if pb is not None and yt.numel() == pb[1] * n:
            # one output per eigen-problem: A = 1/ev and ytilde * A in ONE launch (fgp_inv_eig) instead of
            # the torch chain of get_inv_log_det; Re(A) kept for post_var's quadratic form
            self._task_scalar()
            lam = self.get_lam(0, 0, n).reshape(pb[1], n).contiguous()
            rows = yt.reshape(pb[1], n)
            want = torch.complex128 if self._FAMILY == ops.LATTICE else torch.float64
            assert lam.dtype == want and rows.dtype == want and rows.stride(-1) == 1, (lam.dtype, rows.dtype)
            ya = torch.empty_like(lam)
            wa = torch.empty((pb[1], n), dtype=torch.float64, device=self.device)
            raw = self.raw_noise.detach().reshape(-1)
            _native.call("fgp_inv_eig", self._FAMILY, _native.ptr(lam), _native.ptr(rows), rows.stride(0),
                         _native.ptr(raw), 1 if raw.numel() > 1 else 0, pb[1], n.bit_length() - 1,
                         _native.ptr(ya), _native.ptr(wa), _native.stream_ptr(self.device))
            self._cached(("inv_real", n), lambda: wa.reshape(tuple(pb[0]) + (n,)))
            if self._FAMILY == ops.LATTICE:
                return ops.ifftbr_raw(ya, stable=True, real_out=True).reshape(yt.shape)
            return ops.fwht_raw(ya, stable=True).reshape(yt.shape)
        return ops.inverse_mul(self._FAMILY, yt, self._inv(n), real_out=True)

    @property
    def coeffs(self):
        return self._cached(("coeffs", self._nh), self._coeffs_now)

    # ------------------------------------------------------------------ fit
    def fit(self, loss_metric="MLL", iterations=5000, lr=None, optimizer=None, stop_crit_improvement_threshold=5e-2,
            stop_crit_wait_iterations=10, store_hists=False, store_loss_hist=False, store_scale_hist=False,
            store_lengthscales_hist=False, store_noise_hist=False, store_task_kernel_hist=False, verbose=5,
            verbose_indent=4, masks=None, cv_weights=1):
        """Hyper-parameter optimisation with the reference's semantics (abstract_gp.py:152-306)."""
        assert isinstance(loss_metric, str) and loss_metric.upper() in ["MLL", "GCV", "CV"]
        assert self._nh > 0, "cannot fit without data"      # (self.n > 0).any() on the host mirror: no sync
        assert isinstance(iterations, int) and iterations >= 0
        assert (isinstance(verbose, int) or isinstance(verbose, bool)) and verbose >= 0, \
            "require verbose is a non-negative int"
        assert isinstance(verbose_indent, int) and verbose_indent >= 0, \
            "require verbose_indent is a non-negative int"
        assert np.isscalar(stop_crit_improvement_threshold) and 0 < stop_crit_improvement_threshold, \
            "require stop_crit_improvement_threshold is a positive float"
        assert isinstance(stop_crit_wait_iterations, int) and stop_crit_wait_iterations > 0
        assert masks is None or isinstance(masks, torch.Tensor)
        loss_metric = loss_metric.upper()
        hists = dict(loss=store_hists or store_loss_hist,
                     scale=store_hists or (store_scale_hist and self.raw_scale.requires_grad),
                     lengthscales=store_hists or (store_lengthscales_hist and self.raw_lengthscales.requires_grad),
                     noise=store_hists or (store_noise_hist and self.raw_noise.requires_grad),
                     task_kernel=store_hists or (store_task_kernel_hist and (
                         self.raw_factor_task_kernel.requires_grad or self.raw_noise_task_kernel.requires_grad)))
        stop = (np.log(1 + stop_crit_improvement_threshold), stop_crit_wait_iterations)
        if masks is not None and optimizer is None and loss_metric == "MLL" and self._fused_ok():
            mk = self._masked_ysq(masks)
            if mk is not None:
                # only the outputs y[..., *masks] in the loss, shared hyper-parameters: the device fit on their
                # Y = sum |ytilde_b|^2 with d_out = the selected count (abstract_gp.py:220-235, 253-260)
                return self._fit_fused(iterations, 1e-1 if lr is None else lr, stop, hists, verbose, verbose_indent,
                                       ysq=mk[0], d_out=mk[1])
        fused = optimizer is None and masks is None and self._fused_ok() and (
            loss_metric == "MLL" or self._alt_loss_ok(loss_metric, cv_weights))
        if optimizer is None:
            optimizer = None if fused else self.get_default_optimizer(lr)
        else:
            assert isinstance(optimizer, torch.optim.Optimizer)
        if fused:
            return self._fit_fused(iterations, 1e-1 if lr is None else lr, stop, hists, verbose, verbose_indent,
                                   loss_metric=loss_metric, cv_weight=float(cv_weights) if loss_metric == "CV" else 1.0)
        return self._fit_generic(loss_metric, iterations, optimizer, stop, hists, verbose, verbose_indent, masks,
                                 cv_weights)

    def _fused_ok(self):
        # (the adaptive nugget of ONE task is the plain one: noise |tr_00 / tr_00| = noise, util.py:286-290 -- the
        # trace sqrt(n) sum_k lambda_k = n k1[0] > 0 for these positive kernels)
        n = self._nh
        if n < 16 or self.d > 8:
            return False
        if self._tfs["scale"][1] is not _exp or self._tfs["lengthscales"][1] is not _exp or \
                self._tfs["noise"][1] is not _exp:
            return False
        if self.raw_factor_task_kernel.requires_grad or self.raw_noise_task_kernel.requires_grad:
            return False
        if not self._task_unit():
            return False
        pb = self._problem_batch()
        return pb is not None

    def _alt_loss_ok(self, loss_metric, cv_weights):
        """fit(loss_metric="GCV" / "CV") on the device (fgp_nll_desc.loss_metric, ABI 16): the spectral path
        (d <= 6), one loss over at most 16 eigen-problems, a scalar cv_weights (the Parseval form of CV's
        sum_i (coeffs_i / inv_diag)^2 w needs one weight for every point); FGP_ALT_LOSS_DEVICE=0 keeps the generic
        autograd loop (A/B, tests)."""
        if os.environ.get("FGP_ALT_LOSS_DEVICE", "1")[:1] == "0" or self.d > SPEC_MAX_D:
            return False
        if loss_metric == "CV":
            if torch.is_tensor(cv_weights):
                if cv_weights.numel() != 1:
                    return False
            elif not np.isscalar(cv_weights):
                return False
        pb = self._problem_batch()
        return pb is not None and pb[1] <= 16 and self._spec_basis(self._nh, pb[1], force=True) is not None

    def _masked_ysq(self, masks):
        """(Y [1, n], d_out) of fit(masks=...) with ONE eigen-problem (hyper-parameters shared by the outputs): Y sums
        |ytilde_b|^2 over the selected outputs y[..., *masks] (repeats counted, as the reference's indexing does) and d_out
        is their count (abstract_gp.py:220-224; the logdet term then weighs the shared logdet d_out times, :258-259).
        None when the problem batch has several eigen-problems (per-output hyper-parameters: the generic path)."""
        pb = self._problem_batch()
        if pb is None or pb[1] != 1 or len(self.shape_batch) == 0:
            return None
        masks = torch.atleast_2d(masks)
        assert masks.ndim == 2 and len(masks) <= len(self.shape_batch)
        d_out = torch.empty(self.shape_batch)[(..., *masks)].numel()
        n = self._nh
        half = self._ytilde_half()
        idx = tuple(m.to(self.device) for m in masks)
        if half is not None:
            sel = half[(..., *idx, slice(None))]
            return ops.sum_sq_half(sel.reshape(-1, sel.shape[-1]).contiguous(), n, 1), d_out
        yt = self.get_ytilde(0)
        sel = yt[(..., *idx, slice(None))]
        return ops.sum_sq(sel.reshape(-1, n).contiguous(), 1), d_out

    def _problem_batch(self):
        """G and the per-problem flags for the fused layout (None when shapes need broadcasting)."""
        shapes = [self.raw_scale.shape[:-1], self.raw_lengthscales.shape[:-1], self.raw_noise.shape[:-1]]
        big = max(shapes, key=len)
        G = math.prod(big)
        for s in shapes:
            cnt = math.prod(s)
            if cnt != 1 and s != big:
                return None
        return big, G

    def _ysq(self, pb_shape, G):
        """Y[g] = sum over the outputs of problem g of |ytilde|^2 (fgp_sum_sq, one pass over ytilde; over its
        Hermitian half -- fgp_sum_sq_half, the same values -- when only that exists)."""
        half = self._ytilde_half()
        if half is not None:
            return ops.sum_sq_half(half.reshape(-1, half.shape[-1]), self._nh, G)
        yt = self.get_ytilde(0)
        return ops.sum_sq(yt.reshape(-1, yt.shape[-1]), G)

    def _log_header(self, verbose, indent):
        if verbose:
            s = "%16s | %-10s | %-10s | %-10s" % ("iter of %.1e" % self._iters_for_log, "loss", "term1", "term2")
            print(" " * indent + s)
            print(" " * indent + "~" * len(s))

    def _log_row(self, i, loss, t1, t2, indent):
        print(" " * indent + "%16.2e | %-10.2e | %-10.2e | %-10.2e" % (i, loss, t1, t2))

    def _fused_engine(self, iterations, lr, ysq=None, d_out=None, loss_metric="MLL", cv_weight=1.0):
        """The FusedMLL of this GP's fit: G eigen-problems from the part-product spectra, the regenerated
        lattice parts or the parts array; `ysq` / `d_out` override Y = sum_b |ytilde_b|^2 and the output
        count (distributed.fit_sharded: Y all-reduced over the ranks' output shards); loss_metric GCV / CV: the
        spectral path's alternative losses (FusedMLL)."""
        n = self._nh
        pb_shape, G = self._problem_batch()
        if d_out is None:
            d_out = math.prod(self.shape_batch)
        basis = self._spec_basis(n, G, force=loss_metric != "MLL")
        gen = self._parts_gen(n) if basis is None else None
        parts = self._k1parts(n) if (gen is None and basis is None) else None
        ls_raw = self.raw_lengthscales.detach()
        ls2 = ls_raw.reshape(-1, ls_raw.shape[-1])
        max_iters = iterations + 1 if G == 1 and iterations < 8192 else min(iterations + 1, 64)
        rg = (self.raw_scale.requires_grad, self.raw_lengthscales.requires_grad, self.raw_noise.requires_grad)
        if basis is not None:
            # the spectral fit's engine, reused across fit() calls of this geometry (fit_engine.cached_engine)
            return cached_engine(self._FAMILY, self._ysq(pb_shape, G) if ysq is None else ysq,
                                 self.raw_scale.detach().reshape(-1), ls2, self.raw_noise.detach().reshape(-1),
                                 logdet_weight=d_out / G, mll_const=mll_constant(d_out, n), requires_grad=rg, lr=lr,
                                 max_iters=max_iters, basis=basis, loss_metric=loss_metric, cv_weight=cv_weight)
        return FusedMLL(self._FAMILY, parts, self._ysq(pb_shape, G) if ysq is None else ysq,
                        self.raw_scale.detach().reshape(-1), ls2,
                        self.raw_noise.detach().reshape(-1), logdet_weight=d_out / G,
                        mll_const=mll_constant(d_out, n),
                        requires_grad=(self.raw_scale.requires_grad, self.raw_lengthscales.requires_grad,
                                       self.raw_noise.requires_grad),
                        lr=lr, max_iters=max_iters, gen=gen, basis=basis, loss_metric=loss_metric, cv_weight=cv_weight)

    def _fit_fused(self, iterations, lr, stop, hists, verbose, indent, ysq=None, d_out=None, loss_metric="MLL",
                   cv_weight=1.0):
        """Device-resident fit (the engine of _fused_engine; the reference's loop semantics: loss history, early
        stopping, best iterate) of the MLL, or of the GCV / CV loss (abstract_gp.py:242-273, whose history holds
        the loss itself where the MLL's holds -loss)."""
        logtol, wait_max = stop
        eng = (self._fused_engine(iterations, lr, ysq, d_out) if loss_metric == "MLL" else
               self._fused_engine(iterations, lr, ysq, d_out, loss_metric=loss_metric, cv_weight=cv_weight))
        self._iters_for_log = iterations
        self._log_header(verbose, indent)
        best, save, waited = math.inf, math.inf, 0
        best_i, i, i0, chunk = 0, 0, 0, 4
        total = iterations + 1
        done = False
        losses = []
        persist = getattr(eng, "persist_ok", lambda: False)()
        if persist and not verbose and not any(hists.values()):
            # the whole fit in one launch (fgp_fit_persist), which leaves the best iterate in the engine's raw
            # parameters (ABI 18): they are restored while the launch runs, and the control word is read after
            # that (the host work overlaps the fit instead of following it)
            ip = eng.run_persist(iterations, logtol, wait_max, defer=True)
            if ip is not None:
                self._restore_best(eng, eng.raw)
                if ip < 0:
                    ip = eng.persist_result()
                if ip is not None:
                    eng.release_inputs()
                    return {"iterations": ip}
            persist = False       # a barrier give-up restored the entry state: the launch per iteration below
        if persist:
            # the whole fit in one launch (fgp_fit_persist: the early-stopping rule on the device); the last
            # iteration and the failure word are read back.  A barrier give-up (None) restored the entry state:
            # the fit then runs below on the launch per iteration (the same trajectory bit for bit).
            no_stop = wait_max > iterations
            ip = eng.run_persist(iterations, logtol, wait_max)
            if ip is not None:
                i = ip
                done = True
                if no_stop:
                    l0 = eng.loss_hist[:total, 0, 0]
                    best_i = torch.where(torch.isnan(l0), torch.full_like(l0, math.inf), l0).argmin()
                if not no_stop or verbose or hists["loss"]:
                    rows = eng.loss_hist[:i + 1, 0].cpu().tolist()
                    for r, row in enumerate(rows):
                        lv = float(row[0])
                        losses.append((lv, float(row[1]), float(row[2])))
                        if lv < best and not no_stop:
                            best, best_i = lv, r
                        if verbose and (r % verbose == 0 or r == i):
                            self._log_row(r, lv, row[1], row[2], indent)
        if not done and wait_max > iterations:
            # no early stop is possible: every iteration runs, the best iterate is the first minimum of
            # the loss history (the host rule `lv < best`; NaN never best), found on the device -- one
            # enqueue, no host sync unless losses are logged or returned
            eng.run(0, total, final_no_update=True)
            lh_dev = eng.loss_hist[:total, 0]
            l0 = lh_dev[:, 0]
            best_i = torch.where(torch.isnan(l0), torch.full_like(l0, math.inf), l0).argmin()
            i = iterations
            done = True
            if verbose or hists["loss"]:
                losses = [tuple(r) for r in lh_dev.cpu().tolist()]
                for r in range(total):
                    if verbose and (r % verbose == 0 or r == iterations):
                        self._log_row(r, losses[r][0], losses[r][1], losses[r][2], indent)
        while not done:
            k = min(chunk, total - i0)
            eng.run(i0, k, final_no_update=(i0 + k == total))
            lh = eng.loss_hist[i0:i0 + k, 0].cpu()
            for r in range(k):
                i = i0 + r
                lv = float(lh[r, 0])
                losses.append((lv, float(lh[r, 1]), float(lh[r, 2])))
                if lv < best:
                    best, best_i = lv, i
                if (save - lv) > logtol:
                    waited = 0
                    save = best
                else:
                    waited += 1
                brk = i == iterations or waited == wait_max
                if verbose and (i % verbose == 0 or brk):
                    self._log_row(i, lv, losses[-1][1], losses[-1][2], indent)
                if brk:
                    done = True
                    break
            i0 += k
            chunk = min(64, chunk * 2)
        raw_hist = eng.raw_hist[:i + 1]
        s_raw, l_raw, nz_raw = eng.split_raw(raw_hist)
        # (a device index tensor: index_select, not raw_hist[t] -- a 0-d index tensor is read back to the host)
        best_row = raw_hist.index_select(0, best_i.reshape(1))[0] if torch.is_tensor(best_i) else raw_hist[best_i]
        self._restore_best(eng, best_row)
        if hasattr(eng, "release_inputs"):
            eng.release_inputs()
        data = {"iterations": i}
        if hists["loss"]:
            sgn = -1.0 if loss_metric == "MLL" else 1.0        # metric_val: -loss (MLL), loss (GCV, CV)
            data["loss_hist"] = torch.tensor([sgn * v[0] for v in losses])
        if hists["scale"]:
            data["scale_hist"] = self.tf_scale(s_raw.reshape((-1,) + self.raw_scale.shape)).cpu()
        if hists["lengthscales"]:
            data["lengthscales_hist"] = self.tf_lengthscales(l_raw.reshape((-1,) + self.raw_lengthscales.shape)).cpu()
        if hists["noise"]:
            data["noise_hist"] = self.tf_noise(nz_raw.reshape((-1,) + self.raw_noise.shape)).cpu()
        if hists["task_kernel"]:
            tkr = eng.task_kernel_rows(raw_hist) if hasattr(eng, "task_kernel_rows") else None
            if tkr is not None:
                data["task_kernel_hist"] = tkr.detach().cpu()
            else:
                data["task_kernel_hist"] = self.gram_matrix_tasks.detach().cpu()[None].expand(
                    (i + 1,) + self.gram_matrix_tasks.shape).clone()
        return data

    def _restore_best(self, eng, best_row):
        """The best iterate's raw parameters (a device row of the engine's layout) as this GP's Parameters
        (abstract_gp.py:285-296), the hyper-parameter-dependent caches dropped."""
        b_s, b_l, b_n = eng.split_raw(best_row)
        restore = [("raw_scale", b_s), ("raw_lengthscales", b_l), ("raw_noise", b_n)]
        tsk = eng.split_task(best_row) if hasattr(eng, "split_task") else None
        if tsk is not None:                             # a multitask engine that also learns the task kernel
            b_f, b_v = tsk
            restore += [("raw_factor_task_kernel", b_f), ("raw_noise_task_kernel", b_v)]
        params = self._parameters
        with torch.no_grad():
            for name, val in restore:
                old = params[name]
                params[name] = torch.nn.Parameter(val.reshape(old.shape).clone(), requires_grad=old.requires_grad)
        self._cache = {k: v for k, v in self._cache.items() if not k[2]}    # keep data-only entries (ytilde, spectra)
        self._snap = None

    def _loss_generic(self, loss_metric, masks, cv_weights, d_out):
        n = self._nh
        A, logdet = self.get_inv_log_det(n)
        A = A[..., 0, 0, :]
        yt = self.get_ytilde(0)
        if loss_metric == "MLL":
            z = yt * A
            norm = (yt.conj() * z).real.sum(-1, keepdim=True) if yt.is_complex() else (yt * z).sum(-1, keepdim=True)
            logdet = logdet[..., None]
            if masks is None:
                t1 = norm.sum()
                t2 = d_out / torch.tensor(logdet.shape).prod() * logdet.sum()
            else:
                t1 = norm[(..., *masks, 0)].sum()
                t2 = logdet.expand(list(self.shape_batch) + [1])[(..., *masks, 0)].sum()
            return 0.5 * (t1 + t2 + d_out * n * np.log(2 * np.pi)), t1, t2, None
        if loss_metric == "GCV":
            z = yt * A
            numer = (z.conj() * z).real.sum(-1, keepdim=True) if z.is_complex() else (z * z).sum(-1, keepdim=True)
            denom = ((A.real if A.is_complex() else A).sum(-1, keepdim=True) / n) ** 2
            if masks is None:
                t1, t2 = numer, denom
            else:
                t1 = numer[(..., *masks, slice(None))]
                t2 = denom.expand(list(self.shape_batch) + [1])[(..., *masks, slice(None))]
            loss = (t1 / t2).sum()
            return loss, t1, t2, loss
        # CV (util.py:381-385 single task; abstract_gp.py:262-273)
        coeffs = self._solve(self._y[0], n)
        lam = self.get_lam(0, 0, n)
        inv_diag = (1 / (lam * np.sqrt(n))).mean(-1, keepdim=True)
        sq = ((coeffs / inv_diag) ** 2 * cv_weights)
        sq = (sq.real if sq.is_complex() else sq).sum(-1, keepdim=True)
        loss = sq.sum() if masks is None else sq[(..., *masks, 0)].sum()
        nan = torch.nan * torch.ones(1)
        return loss, nan, nan, loss

    def _fit_generic(self, loss_metric, iterations, optimizer, stop, hists, verbose, indent, masks, cv_weights):
        logtol, wait_max = stop
        if masks is not None:
            masks = torch.atleast_2d(masks)
            assert masks.ndim == 2 and len(masks) <= len(self.shape_batch)
            d_out = torch.empty(self.shape_batch)[(..., *masks)].numel()
        else:
            d_out = int(torch.tensor(self.shape_batch).prod())
        self._iters_for_log = iterations
        self._log_header(verbose, indent)
        rec = {k: [] for k in ("loss", "scale", "lengthscales", "noise", "task_kernel")}
        best, save, waited = math.inf, math.inf, 0
        best_params = None
        for i in range(iterations + 1):
            self._cache = {k: v for k, v in self._cache.items() if not k[2]}
            loss, t1, t2, metric = self._loss_generic(loss_metric, masks, cv_weights, d_out)
            lv = loss.item()
            if lv < best:
                best = lv
                best_params = {k: p.data.clone() for k, p in self.named_parameters()}
            if (save - lv) > logtol:
                waited = 0
                save = best
            else:
                waited += 1
            brk = i == iterations or waited == wait_max
            if hists["loss"]:
                rec["loss"].append(-lv if metric is None else metric.item())
            if hists["scale"]:
                rec["scale"].append(self.scale.detach().cpu())
            if hists["lengthscales"]:
                rec["lengthscales"].append(self.lengthscales.detach().cpu())
            if hists["noise"]:
                rec["noise"].append(self.noise.detach().cpu())
            if hists["task_kernel"]:
                rec["task_kernel"].append(self.gram_matrix_tasks.detach().cpu())
            if verbose and (i % verbose == 0 or brk):
                self._log_row(i, lv, t1.item() if t1.numel() == 1 else torch.nan,
                              t2.item() if t2.numel() == 1 else torch.nan, indent)
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
        if hists["loss"]:
            data["loss_hist"] = torch.tensor(rec["loss"])
        for k in ("scale", "lengthscales", "noise", "task_kernel"):
            if hists[k]:
                data[k + "_hist"] = torch.stack(rec[k])
        return data

    # ------------------------------------------------------------------ prediction
    def _hyp_rows(self, batch_params):
        """[Gk, 1+d] (scale, lengthscales) rows for the prediction kernels (cached per parameters)."""
        return self._cached(("hyp_rows", bool(batch_params)), lambda: self._hyp_rows_now(batch_params))

    def _hyp_rows_now(self, batch_params):
        s, ls = self.scale.detach(), self.lengthscales.detach()
        if not batch_params:
            return torch.cat([s.reshape(1), ls.reshape(-1).expand(self.d)])[None]
        sb = self.shape_batch
        s = s.expand(tuple(sb) + (1,)).reshape(-1, 1)
        ls = ls.expand(tuple(sb) + (self.d,)).reshape(-1, self.d)
        return torch.cat([s, ls], -1)

    def _has_batch_params(self):
        return self.raw_scale.dim() > 1 or self.raw_lengthscales.dim() > 1

    def _check_unit(self, x, name="x"):
        assert ((0 <= x) & (x <= 1)).all(), "%s should have all elements in [0,1]" % name

    def _defer_unit(self, x, name="x"):
        """Enqueue the [0, 1] range check of x (fast_gp_lattice.py:264-265) without synchronising;
        _raise_deferred() reads all pending flags back once, after the dependent work is enqueued.
        A tensor already checked (same storage, version counter, shape and strides) is not re-checked."""
        key = (x.data_ptr(), x._version, tuple(x.shape), tuple(x.stride()), x.device)
        if any(k == key for k, _ in getattr(self, "_unit_ok", ())):
            return
        flag = ((0 <= x) & (x <= 1)).all()
        self._pending_checks = getattr(self, "_pending_checks", []) + [(flag, name, (key, x))]

    def _raise_deferred(self):
        pend = getattr(self, "_pending_checks", [])
        self._pending_checks = []
        if pend:
            ok = torch.stack([f for f, _, _ in pend]).cpu()
            for good, (_, name, _) in zip(ok.tolist(), pend):
                assert good, "%s should have all elements in [0,1]" % name
            # (the checked tensors are held, so their storage cannot be reused under the same key)
            seen = getattr(self, "_unit_ok", [])
            self._unit_ok = (seen + [kx for _, _, kx in pend])[-8:]

    def _task_arg(self, task):
        if task is None:
            task = self.default_task
        inttask = isinstance(task, int)
        if inttask:
            task = torch.tensor([task], dtype=torch.int64)
        if isinstance(task, list):
            task = torch.tensor(task, dtype=torch.int64)
        assert task.ndim == 1 and (task >= 0).all() and (task < self.num_tasks).all()
        return inttask

    def _n_arg(self, n):
        if n is None:
            return self._nh       # host mirror of self.n: no device round trip
        if isinstance(n, (int, np.integer)):
            n = int(n)
            assert n > 0 and (n & (n - 1)) == 0 and n >= self._nh, \
                "require n are all power of two greater than or equal to self.n"
            return n
        if isinstance(n, int):
            n = torch.tensor([n], dtype=torch.int64, device=self.device)
        assert isinstance(n, torch.Tensor) and (n & (n - 1) == 0).all() and (n >= self.n).all(), \
            "require n are all power of two greater than or equal to self.n"
        return int(n.reshape(-1)[0])

    def _cross_rows(self, x, n, batch_params):
        """rows[g, t, i] = K(x_t, xb_i) for the first n points."""
        z = self._points_T(n)
        return ops.kernel_rows(self._FAMILY, x, z, self._hyp_rows(batch_params), alphas=self._alphas,
                               tbits=self._tbits())

    def _post_var_qf(self, x, n, chunk=16):
        """sum_k Re(A_k) |ft(K(x_t, .))_k|^2 for every test point (fgp_post_var_qf)."""
        z = self._points_T(n)

        def real_inv():
            wa = self._inv(n)
            return (wa.real if wa.is_complex() else wa).contiguous()
        wa = self._cached(("inv_real", n), real_inv)
        hyp = self._hyp_rows(False)[0].contiguous()
        out = torch.empty(x.size(0), dtype=torch.float64, device=self.device)
        for t0 in range(0, x.size(0), chunk):
            xs = x[t0:t0 + chunk].contiguous()
            out[t0:t0 + xs.size(0)] = ops.post_var_quadform(self._FAMILY, xs, z, hyp, wa, alphas=self._alphas,
                                                            tbits=self._tbits())
        return out

    def _post_var_problems(self, x, n, work_bytes=1 << 30):
        """Per-problem hyper-parameters (G eigen-problems on one point set, e.g. C5 per-output): every
        problem's quadratic form sum_k Re(A_gk) |ft(K_g(x_t, .))_k|^2 and K_g(x, x) by
        fgp_post_var_batched (shared points, z_stride 0), problems in chunks of <= work_bytes scratch --
        instead of G x N kernel rows solved by full-length transforms."""
        pb, G = self._problem_batch()
        out = self._post_var_spectral(x, n, G)
        if out is not None:
            return out.reshape(tuple(self.shape_batch) + (x.size(0),))
        wa = self._cached(("inv_real", n), lambda: (lambda a: (a.real if a.is_complex() else a))(self._inv(n)))
        wa = wa.reshape(G, n).contiguous()
        hyp = self._hyp_rows(True).contiguous()                   # [G, 1 + d]
        z = self._points_T(n)
        order, coef = ops._pred_args(self._FAMILY, self._alphas, self.d)
        x = x.contiguous()
        Nt = x.size(0)
        cdt = torch.complex128 if self._FAMILY == ops.LATTICE else torch.float64
        per = Nt * n * (16 if self._FAMILY == ops.LATTICE else 8)
        pc = max(1, min(G, work_bytes // per))
        work = torch.empty((pc, Nt, n), dtype=cdt, device=self.device)
        partial = torch.empty((pc, Nt, max(1, n >> 12)), dtype=torch.float64, device=self.device)
        out = torch.empty((G, Nt), dtype=torch.float64, device=self.device)
        part0 = _native.double_array([float(v) for v in self._part_at_zero()])
        for p0 in range(0, G, pc):
            p1 = min(G, p0 + pc)
            desc = _native.PredDesc(family=self._FAMILY, d=self.d, tbits=int(self._tbits()), P=p1 - p0, n=n,
                                    z=z.data_ptr(), z_stride=0, hyp=hyp[p0].data_ptr(), hyp_stride=hyp.stride(0),
                                    coeffs=wa[p0].data_ptr(), coeff_stride=n, wa=wa[p0].data_ptr(), wa_stride=n)
            for j in range(self.d):
                desc.order[j] = order[j]
                desc.coef[j] = coef[j]
            _native.call("fgp_post_var_batched", desc, _native.ptr(x), 0, Nt, part0, _native.ptr(out[p0:p1]),
                         _native.ptr(work), _native.ptr(partial), _native.stream_ptr(self.device))
        return out.reshape(tuple(self.shape_batch) + (Nt,))

    def _post_var_spectral(self, x, n, G):
        """[G, N] posterior variances of G lattice eigen-problems on one point set from the row spectra of
        the test points (fgp_spec_post_var): Psi_S(t) = ft(prod_{j in S} part_j(x_t, .)) -- 2^d N transforms
        once, hyper-parameter free -- and ft(K_g(x_t, .)) = scale_g sum_S l_g^S Psi_S(t) by linearity, instead
        of one transform per (problem, test point).  None when it does not apply (nets, d > 4, no shared
        spectra, adaptive nugget, non-exp transforms, or fewer than 16 problems: the per-row transforms are
        then as cheap)."""
        if (self._FAMILY != ops.LATTICE or self.d > 4 or G < 16 or self.adaptive_nugget or not self._lam_fusable(n)
                or os.environ.get("FGP_SPEC_POST_VAR", "1") == "0"):
            return None
        basis = self._spec_basis(n, G)
        if basis is None or basis.dim() != 3:
            return None
        self._task_scalar()
        d, Nt = self.d, x.size(0)
        self._ensure_points(n)
        xb = self._xb[:n]
        # test points in slices: fgp_spec_post_var takes at most SPEC_POST_VAR_MAX_N points per call, and the
        # row products rho [Nt, 2^d, n] float64 + their spectra psi complex128 (24 2^d n bytes per point) stay
        # within SPEC_POST_VAR_WORK bytes
        per = max(1, min(SPEC_POST_VAR_MAX_N, SPEC_POST_VAR_WORK // (24 * (2 ** d) * n)))
        raws = (self.raw_scale.detach().reshape(-1), self.raw_lengthscales.detach().reshape(-1, self.raw_lengthscales.shape[-1]),
                self.raw_noise.detach().reshape(-1))
        part0 = self._part_at_zero().tolist()
        outs = []
        for t0 in range(0, Nt, per):
            xs = x[t0:t0 + per]
            Nc = xs.size(0)
            parts = torch.stack([ops.lattice_parts(xb, xs[t], self._alphas) for t in range(Nc)])   # [Nc, d, n]
            rho = torch.empty((Nc, 2 ** d, n), dtype=torch.float64, device=self.device)
            rho[:, 0] = 1.0
            for S in range(1, 2 ** d):
                j = S.bit_length() - 1
                torch.mul(rho[:, S ^ (1 << j)], parts[:, j], out=rho[:, S])
            del parts
            psi = ops.fftbr_raw(rho, stable=True)
            del rho
            outs.append(spec_post_var(*raws, G, n, basis, psi.contiguous(), part0))
            del psi
        return torch.cat(outs, 1)

    def _kdiag(self, x):
        """K(x, x) (zero distance parts)."""
        part0 = getattr(self, "_part0_dev", None)
        if part0 is None:
            part0 = self._part0_dev = self._part_at_zero().to(self.device)
        return self.scale * (1 + self.lengthscales * part0).prod(-1, keepdim=True)

    def post_mean(self, x, task=None, eval=True):
        """Posterior mean (abstract_gp.py:352-380) via the matrix-free HIP contraction."""
        if eval:
            with torch.no_grad():
                coeffs = self.coeffs
        else:
            coeffs = self.coeffs
        if eval:
            incoming = torch.is_grad_enabled()
            torch.set_grad_enabled(False)
        try:
            assert x.ndim == 2 and x.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
            inttask = self._task_arg(task)
            x = x.to(device=self.device, dtype=torch.float64)
            self._defer_unit(x)
            n = self._nh
            if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
                kmat = self._kernel_torch(x[:, None, :], self._xb[:n][None, :, :])
                pm = torch.einsum("...i,...i->...", kmat, coeffs[..., None, :])
            else:
                bp = self._has_batch_params()
                c2 = coeffs.reshape(-1, n)
                z = self._points_T(n)
                pm = ops.post_mean_matfree(self._FAMILY, x, z, self._hyp_rows(bp), c2, alphas=self._alphas,
                                           tbits=self._tbits())
                pm = pm.reshape(tuple(coeffs.shape[:-1]) + (x.size(0),))
            self._raise_deferred()
        finally:
            if eval:
                torch.set_grad_enabled(incoming)
        return pm if inttask else pm[..., None, :]

    def post_var(self, x, task=None, n=None, eval=True):
        """Posterior variance (abstract_gp.py:381-416, abstract_fast_gp.py:41-46)."""
        n = self._n_arg(n)
        assert x.ndim == 2 and x.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
        if eval:
            incoming = torch.is_grad_enabled()
            torch.set_grad_enabled(False)
        try:
            inttask = self._task_arg(task)
            x = x.to(device=self.device, dtype=torch.float64)
            self._defer_unit(x)
            bp = self._has_batch_params()
            qf_ok = not self._gradmode() and 4096 < n <= 2 ** 24 and self.d <= 8 and self._lam_fusable(n)
            if qf_ok and not bp:
                diag = self._kdiag(x) - self._post_var_qf(x, n)
            elif qf_ok and not self.adaptive_nugget and tuple(self._problem_batch()[0]) == tuple(self.shape_batch):
                diag = self._post_var_problems(x, n)
            else:
                rows = self._cross_rows(x, n, bp)                      # [Gk, N, n]
                kmat = rows[0] if not bp else rows.reshape(tuple(self.shape_batch) + rows.shape[1:])
                t = self._solve(kmat.movedim(-2, 0), n).movedim(0, -2)
                diag = self._kdiag(x) - (t * kmat).sum(-1)
            diag = diag.clamp_(min=0)          # (diag[diag < 0] = 0 without a host sync)
            self._raise_deferred()
        finally:
            if eval:
                torch.set_grad_enabled(incoming)
        return diag if inttask else diag[..., None, :]

    def post_cov(self, x0, x1, task0=None, task1=None, n=None, eval=True):
        """Posterior covariance (abstract_gp.py:417-474, abstract_fast_gp.py:47-52)."""
        n_arg = n if n is not None else self.n
        if isinstance(n_arg, int):
            n_arg = torch.tensor([n_arg], dtype=torch.int64, device=self.device)
        assert isinstance(n_arg, torch.Tensor) and (n_arg & (n_arg - 1) == 0).all() and (n_arg >= self.n).all(), \
            "require n are all power of two"
        n = int(n_arg.reshape(-1)[0])
        assert x0.ndim == 2 and x0.size(1) == self.d, "x must a torch.Tensor with shape (-1,d)"
        assert x1.ndim == 2 and x1.size(1) == self.d, "z must a torch.Tensor with shape (-1,d)"
        if eval:
            incoming = torch.is_grad_enabled()
            torch.set_grad_enabled(False)
        try:
            i0 = self._task_arg(task0)
            i1 = self._task_arg(task1)
            x0 = x0.to(device=self.device, dtype=torch.float64)
            x1 = x1.to(device=self.device, dtype=torch.float64)
            equal = torch.equal(x0, x1)
            bp = self._has_batch_params()
            hyp = self._hyp_rows(bp)
            z1 = (x1 if self._FAMILY == ops.LATTICE else self._to_b(x1)).T.contiguous()
            knew = ops.kernel_rows(self._FAMILY, x0, z1, hyp, alphas=self._alphas, tbits=self._tbits())
            k1 = self._cross_rows(x0, n, bp)
            k2 = k1 if equal else self._cross_rows(x1, n, bp)
            shp = (lambda r: r[0]) if not bp else (lambda r: r.reshape(tuple(self.shape_batch) + r.shape[1:]))
            knew, k1, k2 = shp(knew), shp(k1), shp(k2)
            t = self._solve(k2.movedim(-2, 0), n).movedim(0, -2)    # [..., M, n]
            cov = knew - torch.einsum("...ni,...mi->...nm", k1, t)
            if equal:
                dg = cov.diagonal(dim1=-2, dim2=-1)
                dg[dg < 0] = 0
        finally:
            if eval:
                torch.set_grad_enabled(incoming)
        if i0 and i1:
            return cov
        if i0:
            return cov[..., None, :, :]
        if i1:
            return cov[..., None, :, :]
        return cov[..., None, None, :, :]

    def post_error(self, x, task=None, n=None, confidence=0.99, eval=True):
        assert np.isscalar(confidence) and 0 < confidence < 1, "confidence must be between 0 and 1"
        q = scipy.stats.norm.ppf(1 - (1 - confidence) / 2)
        pvar = self.post_var(x, task=task, n=n, eval=eval)
        return pvar, q, q * torch.sqrt(pvar)

    def post_ci(self, x, task=None, confidence=0.99, eval=True):
        assert np.isscalar(confidence) and 0 < confidence < 1, "confidence must be between 0 and 1"
        q = scipy.stats.norm.ppf(1 - (1 - confidence) / 2)
        pmean = self.post_mean(x, task=task, eval=eval)
        pvar, q, perror = self.post_error(x, task=task, confidence=confidence)
        # the reference scales by q twice (abstract_gp.py:497-498,523-525); kept for drop-in parity
        return pmean, pvar, q, pmean - q * perror, pmean + q * perror

    def post_cubature_mean(self, task=None, eval=True):
        """abstract_fast_gp.py:65-81 (single task)."""
        coeffs = self.coeffs
        if eval:
            incoming = torch.is_grad_enabled()
            torch.set_grad_enabled(False)
        try:
            inttask = self._task_arg(task)
            pc = (self.scale * coeffs).sum(-1) * self._task_scalar()
        finally:
            if eval:
                torch.set_grad_enabled(incoming)
        return pc if inttask else pc[..., None]

    def post_cubature_var(self, task=None, n=None, eval=True):
        """abstract_fast_gp.py:82-109 (single task: the frequency-0 entry of the inverse)."""
        n = self._n_arg(n)
        A = self._inv(n)
        if eval:
            incoming = torch.is_grad_enabled()
            torch.set_grad_enabled(False)
        try:
            inttask = self._task_arg(task)
            term = n * A[..., 0:1]
            term = term.real if term.is_complex() else term
            pcvar = self.scale - self.scale ** 2 * term
            pcvar[pcvar < 0] = 0.
        finally:
            if eval:
                torch.set_grad_enabled(incoming)
        return pcvar[..., 0] if inttask else pcvar

    def post_cubature_cov(self, task0=None, task1=None, n=None, eval=True):
        pv = self.post_cubature_var(task=0, n=n, eval=eval)
        i0 = task0 is None or isinstance(task0, int)
        i1 = task1 is None or isinstance(task1, int)
        if i0 and i1:
            return pv
        return pv[..., None, None] if not (i0 or i1) else pv[..., None]

    def post_cubature_error(self, task=None, n=None, confidence=0.99, eval=True):
        assert np.isscalar(confidence) and 0 < confidence < 1, "confidence must be between 0 and 1"
        q = scipy.stats.norm.ppf(1 - (1 - confidence) / 2)
        pcvar = self.post_cubature_var(task=task, n=n, eval=eval)
        return pcvar, q, q * torch.sqrt(pcvar)

    def post_cubature_ci(self, task=None, confidence=0.99, eval=True):
        assert np.isscalar(confidence) and 0 < confidence < 1, "confidence must be between 0 and 1"
        q = scipy.stats.norm.ppf(1 - (1 - confidence) / 2)
        pcmean = self.post_cubature_mean(task=task, eval=eval)
        pcvar, q, pcerror = self.post_cubature_error(task=task, confidence=confidence, eval=eval)
        return pcmean, pcvar, q, pcmean - pcerror, pcmean + pcerror

    def kernel(self, x, z, beta0=None, beta1=None, c0=None, c1=None):
        """K(x, z) with broadcasting of x [..., d] and z [..., d] (abstract_gp.py:693-706 ->
        abstract_fast_gp.py:192-196).  beta = 0 with unit coefficients: the differentiable torch form of the
        family kernel; derivative multi-indices beta0 [p0, d] / beta1 [p1, d] with coefficients c0 / c1: the
        parts with derivative orders (fgp_mt_parts: lattice Bernoulli order 2 alpha - beta - kappa, net
        (-2)^(beta+kappa) (ind + omega)) combined by _kernel_from_parts (abstract_fast_gp.py:181-191)."""
        assert isinstance(x, torch.Tensor) and x.size(-1) == self.d
        assert isinstance(z, torch.Tensor) and z.size(-1) == self.d
        dev = self.device
        plain = all(b is None or not bool((b != 0).any()) for b in (beta0, beta1)) and \
            all(c is None or (c.numel() == 1 and float(c.reshape(-1)[0]) == 1.0) for c in (c0, c1)) and \
            all(b is None or b.numel() == self.d for b in (beta0, beta1))
        if plain and not self._MULTITASK:
            return self._kernel_torch(x, z)
        if beta0 is None:
            beta0 = torch.zeros((1, self.d), dtype=torch.int64, device=dev)
        if beta0.shape == (len(beta0),):
            beta0 = beta0[None, :]
        assert isinstance(beta0, torch.Tensor) and beta0.ndim == 2 and beta0.size(1) == self.d
        if beta1 is None:
            beta1 = torch.zeros((1, self.d), dtype=torch.int64, device=dev)
        if beta1.shape == (len(beta1),):
            beta1 = beta1[None, :]
        assert isinstance(beta1, torch.Tensor) and beta1.ndim == 2 and beta1.size(1) == self.d
        if c0 is None:
            c0 = torch.ones(len(beta0), device=dev)
        assert isinstance(c0, torch.Tensor) and c0.shape == (beta0.size(0),)
        if c1 is None:
            c1 = torch.ones(len(beta1), device=dev)
        assert isinstance(c1, torch.Tensor) and c1.shape == (beta1.size(0),)
        shape = torch.broadcast_shapes(x.shape[:-1], z.shape[:-1])
        xe = x.expand(shape + (self.d,)).reshape(-1, self.d)
        ze = z.expand(shape + (self.d,)).reshape(-1, self.d)
        p = self._parts_pairs(xe, ze, beta0.cpu(), beta1.cpu(), zip_pairs=True)
        k = self._kernel_from_parts(p, beta0.to(dev), beta1.to(dev), c0.to(dev, torch.float64), c1.to(dev, torch.float64))
        return k.reshape(k.shape[:-1] + tuple(shape))

    # ------------------------------------------------------------------ kernel parts with derivative orders
    def _pair_spec(self, beta0, beta1):
        """(order, coef, add) [p0 p1, d] for fgp_mt_parts (fast_gp_lattice.py:267-273,
        fast_gp_digital_net_b2.py:289-301); coefficients evaluated with the reference's own ops (memoised per
        (beta0, beta1): the multitask pair spectra ask for the same derivative orders pair after pair)."""
        key = (tuple(beta0.shape), tuple(beta0.reshape(-1).tolist()), tuple(beta1.shape),
               tuple(beta1.reshape(-1).tolist()), tuple(self._alphas))
        memo = self.__dict__.setdefault("_pair_spec_memo", {})
        if key not in memo:
            memo[key] = self._pair_spec_eval(beta0, beta1)
        return memo[key]

    def _pair_spec_eval(self, beta0, beta1):
        alpha = torch.tensor(self._alphas, dtype=torch.int64)
        order, coef, add = [], [], []
        for b0 in beta0:
            for b1 in beta1:
                bpk = b0 + b1
                if self._FAMILY == ops.LATTICE:
                    o = 2 * alpha - bpk
                    assert (2 <= o).all(), "order must all be at least 2, but got order = %s" % str(o)
                    c = (-1) ** (alpha + b1 + 1) * torch.exp(2 * alpha * np.log(2 * np.pi) - torch.lgamma(o + 1))
                    a = torch.zeros(self.d)
                else:
                    o = alpha - bpk
                    assert (1 <= o).all() and (o <= 4).all(), \
                        "order must all be between 2 and 4, but got order = %s. Try increasing alpha" % str(o)
                    c = ((-2) ** bpk).to(torch.float64)
                    a = (bpk > 0).to(torch.float64)
                order.append([int(v) for v in o.tolist()])
                coef.append([float(v) for v in c.tolist()])
                add.append([float(v) for v in a.tolist()])
        return order, coef, add

    def _kargs(self, x, check=True):
        """points as the parts kernel takes them: float64 lattice points, int64 t-bit net points.  check: the
        reference's [0, 1] range assertion (fast_gp_lattice.py:264-265; a device->host sync) -- skipped for the
        GP's own point sets (get_xb), which are in range by construction."""
        if self._FAMILY == ops.LATTICE:
            x = x.to(device=self.device, dtype=torch.float64)
            if check:
                assert bool(((0 <= x) & (x <= 1)).all()), "x should have all elements in [0,1]"
            return x
        if torch.is_floating_point(x):
            x = x.to(self.device)
            if check:
                assert bool(((0 <= x) & (x <= 1)).all()), "x should have all elements in [0,1]"
            return torch.floor((x % 1) * 2 ** self.t).to(torch.int64)
        return x.to(device=self.device, dtype=torch.int64)

    def _parts_pairs(self, x, z, beta0, beta1, zip_pairs=False, check=True):
        """_kernel_parts (abstract_fast_gp.py:173-180) for all (x_i, z_k) pairs -> [N, M, p0, p1, d]
        (or the (x_i, z_i) pairs -> [N, p0, p1, d])."""
        order, coef, add = self._pair_spec(beta0, beta1)
        p = ops.mt_parts(self._FAMILY, self._kargs(x, check), self._kargs(z, check), order, coef, add, self._tbits(),
                         zip_pairs)
        return p.reshape(p.shape[:-2] + (len(beta0), len(beta1), self.d))

    def _kernel_from_parts(self, parts, beta0, beta1, c0, c1):
        """abstract_fast_gp.py:181-191."""
        ndim = parts.ndim
        scale = self.scale.reshape(self.scale.shape + torch.Size([1] * (ndim - 2)))
        ls = self.lengthscales
        ls = ls.reshape(ls.shape[:-1] + torch.Size([1] * (ndim - 1) + [ls.size(-1)]))
        ind = ((beta0[:, None, :] + beta1[None, :, :]) == 0).to(torch.int64)
        terms = scale * (ind + ls * parts).prod(-1)
        return ((terms * c1).sum(-1) * c0).sum(-1)


class FastGPLattice(AbstractFastGP):
    """Fast GP on shifted rank-1 lattices with shift-invariant (Bernoulli) kernels: the Gram matrix
    is diagonalised by the bit-reversed-input FFT (fastgps/fast_gp_lattice.py:7-273)."""

    _FAMILY = ops.LATTICE
    _XBDTYPE = torch.float64
    _FTOUTDTYPE = torch.complex128

    def __init__(self, seqs, num_tasks=None, seed_for_seq=None, alpha=2, scale=1., lengthscales=1., noise=1e-8,
                 factor_task_kernel=1., rank_factor_task_kernel=None, noise_task_kernel=1., device="cuda",
                 tfs_scale=_DEFAULT_TFS, tfs_lengthscales=_DEFAULT_TFS, tfs_noise=_DEFAULT_TFS,
                 tfs_factor_task_kernel=_IDENTITY_TFS, tfs_noise_task_kernel=_DEFAULT_TFS, requires_grad_scale=True,
                 requires_grad_lengthscales=True, requires_grad_noise=False, requires_grad_factor_task_kernel=None,
                 requires_grad_noise_task_kernel=None, shape_batch=torch.Size([]), shape_scale=torch.Size([1]),
                 shape_lengthscales=None, shape_noise=torch.Size([1]), shape_factor_task_kernel=None,
                 shape_noise_task_kernel=None, derivatives=None, derivatives_coeffs=None, compile_fts=False,
                 compile_fts_kwargs={}, adaptive_nugget=False, data_dtype=torch.float64):
        assert isinstance(alpha, int) and alpha in (1, 2, 3, 4), "alpha must be in [1, 2, 3, 4]"
        super().__init__(seqs, num_tasks, seed_for_seq, alpha, scale, lengthscales, noise, factor_task_kernel,
                         rank_factor_task_kernel, noise_task_kernel, device, tfs_scale, tfs_lengthscales, tfs_noise,
                         tfs_factor_task_kernel, tfs_noise_task_kernel, requires_grad_scale,
                         requires_grad_lengthscales, requires_grad_noise, requires_grad_factor_task_kernel,
                         requires_grad_noise_task_kernel, shape_batch, shape_scale, shape_lengthscales, shape_noise,
                         shape_factor_task_kernel, shape_noise_task_kernel, derivatives, derivatives_coeffs,
                         compile_fts, compile_fts_kwargs, adaptive_nugget, data_dtype=data_dtype)

    def _default_seq(self, d, seed):
        return _seqs.Lattice(d, seed=seed, randomize="SHIFT")

    def _check_seq(self, s):
        assert getattr(s, "order", "NATURAL") == "NATURAL", "each seq should be in 'NATURAL' order "
        assert getattr(s, "replications", 1) == 1, "each seq should have only 1 replication"
        assert getattr(s, "randomize", "SHIFT") in ["FALSE", "SHIFT"], \
            "each seq should have randomize in ['FALSE','SHIFT']"

    def _sample(self, n_min, n_max):
        return self._sample_seq(self.seq, n_min, n_max)

    def _sample_seq(self, seq, n_min, n_max):
        """Points [n_min, n_max) of a natural-order lattice: on the device (fgp_lattice_points,
        bit-identical to seqs.Lattice) for this package's generator, else from the seq object."""
        if isinstance(seq, _seqs.Lattice) and n_max > n_min:
            z = [int(v) for v in seq.z[:self.d]]
            bits = max(1, int(n_max - 1).bit_length())
            if all(0 < v < 2 ** (53 - bits) for v in z) and np.all((seq.shift >= 0) & (seq.shift < 1)):
                x = ops.lattice_points(z, seq.shift, int(n_min), int(n_max), device=self.device)
                return x, x
        x = torch.from_numpy(np.asarray(seq(n_min=int(n_min), n_max=int(n_max)), dtype=np.float64)).to(self.device)
        return x, x

    def _tbits(self):
        return 0

    def get_omega(self, m):
        return torch.exp(-torch.pi * 1j * torch.arange(2 ** m, device=self.device) / 2 ** m)

    def ft(self, x):
        return ops.fftbr(x, stable=True)

    def ift(self, x):
        return ops.ifftbr(x, stable=True)

    def _compute_parts(self, xb, x0, out=None):
        self._defer_unit(xb)
        parts = ops.lattice_parts(xb, x0, self._alphas, out=out)
        self._raise_deferred()
        return parts

    def _parts_gen(self, n):
        """Regenerate the parts in the fused kernels (FGP_PARTS_LATTICE) when the points are this
        package's natural-order Lattice: bit-identical to the parts array, without its 2 x 8nd bytes of
        HBM reads per fit iteration.  FGP_PARTS_GEN=0 disables it."""
        if os.environ.get("FGP_PARTS_GEN", "1") == "0" or not isinstance(self.seq, _seqs.Lattice):
            return None
        memo = getattr(self, "_pgen_memo", None)      # (a function of the point set and n only)
        if memo is not None and memo[0] == n and memo[1] is self.seq:
            return memo[2]
        gen = self._parts_gen_new(n)
        self._pgen_memo = (n, self.seq, gen)
        return gen

    def _parts_gen_new(self, n):
        m = int(n).bit_length() - 1
        z = [int(v) for v in self.seq.z[:self.d]]
        if len(z) != self.d or not all(0 < v < 2 ** (53 - m) for v in z) or len(set(self._alphas)) != 1:
            return None
        if not np.all((self.seq.shift >= 0) & (self.seq.shift < 1)):
            return None
        self._ensure_points(1)
        return LatticePartsGen(z, self._alphas, self._x[0:1])

    def _part_at_zero(self):
        return torch.tensor([ops.lattice_coefficient(a) * float(_bern(2 * a, 0.0)) for a in self._alphas],
                            dtype=torch.float64)

    def _kernel_torch(self, x, z):
        delta = (x - z) % 1
        parts = torch.stack([ops.lattice_coefficient(a) * _bern_t(2 * a, delta[..., j])
                             for j, a in enumerate(self._alphas)], -1)
        ndim = parts.ndim
        s = self.scale.reshape(self.scale.shape + torch.Size([1] * (ndim - 2)))
        ls = self.lengthscales.reshape(self.lengthscales.shape[:-1] + torch.Size([1] * (ndim - 1)) +
                                       self.lengthscales.shape[-1:])
        return s * (1 + ls * parts).prod(-1)


class FastGPDigitalNetB2(AbstractFastGP):
    """Fast GP on digitally shifted base-2 digital nets with digitally-shift-invariant (Walsh)
    kernels: the Gram matrix is diagonalised by the FWHT (fastgps/fast_gp_digital_net_b2.py:7-301).
    Walsh orders alpha = 1..4 (default 2).  Order 1 follows the reference's inline formula
    (:297-298); orders 2-4 are the series omega_a = sum_{k>=1} 2^(-mu_a(k)) wal_k that the reference
    takes from qmcpy.kernel_methods.weighted_walsh_funcs(a, ., t) - 1 (:300) -- restated here from
    that definition (walsh_omega in csrc/fgp_common.h); qmcpy is absent offline, so parity at that
    boundary is unpinned."""

    _FAMILY = ops.NET
    _XBDTYPE = torch.int64
    _FTOUTDTYPE = torch.float64

    def __init__(self, seqs, num_tasks=None, seed_for_seq=None, alpha=2, scale=1., lengthscales=1., noise=1e-16,
                 factor_task_kernel=1., rank_factor_task_kernel=None, noise_task_kernel=1., device="cuda",
                 tfs_scale=_DEFAULT_TFS, tfs_lengthscales=_DEFAULT_TFS, tfs_noise=_DEFAULT_TFS,
                 tfs_factor_task_kernel=_IDENTITY_TFS, tfs_noise_task_kernel=_DEFAULT_TFS, requires_grad_scale=True,
                 requires_grad_lengthscales=True, requires_grad_noise=False, requires_grad_factor_task_kernel=None,
                 requires_grad_noise_task_kernel=None, shape_batch=torch.Size([]), shape_scale=torch.Size([1]),
                 shape_lengthscales=None, shape_noise=torch.Size([1]), shape_factor_task_kernel=None,
                 shape_noise_task_kernel=None, derivatives=None, derivatives_coeffs=None, compile_fts=False,
                 compile_fts_kwargs={}, adaptive_nugget=False, data_dtype=torch.float64):
        super().__init__(seqs, num_tasks, seed_for_seq, alpha, scale, lengthscales, noise, factor_task_kernel,
                         rank_factor_task_kernel, noise_task_kernel, device, tfs_scale, tfs_lengthscales, tfs_noise,
                         tfs_factor_task_kernel, tfs_noise_task_kernel, requires_grad_scale,
                         requires_grad_lengthscales, requires_grad_noise, requires_grad_factor_task_kernel,
                         requires_grad_noise_task_kernel, shape_batch, shape_scale, shape_lengthscales, shape_noise,
                         shape_factor_task_kernel, shape_noise_task_kernel, derivatives, derivatives_coeffs,
                         compile_fts, compile_fts_kwargs, adaptive_nugget, data_dtype=data_dtype)
        assert (1 <= self.alpha).all() and (self.alpha <= 4).all()
        self.t = int(self.seq.t)
        assert self.t < 64, "each seq must have t<64"

    def _default_seq(self, d, seed):
        return _seqs.DigitalNetB2(d, seed=seed, randomize="DS")

    def _check_seq(self, s):
        assert getattr(s, "order", "NATURAL") == "NATURAL", "each seq should be in 'NATURAL' order "
        assert getattr(s, "replications", 1) == 1, "each seq should have only 1 replication"
        assert getattr(s, "randomize", "DS") in ['FALSE', 'DS', 'LMS', 'LMS_DS'], \
            "seq should have randomize in ['FALSE','DS','LMS','LMS_DS']"

    def _sample(self, n_min, n_max):
        return self._sample_seq(self.seq, n_min, n_max)

    def _sample_seq(self, seq, n_min, n_max):
        """Points [n_min, n_max) of a natural-order digital net: on the device (fgp_net_points,
        generating-matrix XOR, bit-identical to seqs.DigitalNetB2) for this package's generator, else from
        the seq object (qmcpy's return_binary=True interface)."""
        if isinstance(seq, _seqs.DigitalNetB2) and n_max > n_min and int(n_max - 1).bit_length() <= seq.C.shape[1]:
            return ops.net_points(seq.C, seq.shift, seq.t, int(n_min), int(n_max), self.device)
        xb = torch.from_numpy(np.asarray(seq(n_min=int(n_min), n_max=int(n_max), return_binary=True))
                              .astype(np.int64)).to(self.device)
        return self._convert_from_b(xb), xb

    def _tbits(self):
        return self.t

    def get_omega(self, m):
        return 1

    def _to_b(self, x):
        return torch.floor((x % 1) * 2 ** self.t).to(torch.int64)

    _convert_to_b = _to_b

    def _convert_from_b(self, xb):
        return xb * 2 ** (-self.t)

    def ft(self, x):
        return ops.fwht(x, stable=True)

    def ift(self, x):
        return ops.fwht(x, stable=True)

    def _compute_parts(self, xb, x0, out=None):
        return ops.net_parts(xb, x0, self.t, out=out, alphas=self._alphas)

    def _part_at_zero(self):
        return torch.tensor([_WALSH_AT_ZERO[a] for a in self._alphas], dtype=torch.float64)

    def _kernel_torch(self, x, z):
        xb = self._to_b(x) if torch.is_floating_point(x) else x
        zb = self._to_b(z) if torch.is_floating_point(z) else z
        delta = xb ^ zb
        parts = torch.stack([walsh_part_t(a, delta[..., j], self.t) for j, a in enumerate(self._alphas)], -1)
        ndim = parts.ndim
        s = self.scale.reshape(self.scale.shape + torch.Size([1] * (ndim - 2)))
        ls = self.lengthscales.reshape(self.lengthscales.shape[:-1] + torch.Size([1] * (ndim - 1)) +
                                       self.lengthscales.shape[-1:])
        return s * (1 + ls * parts).prod(-1)


# omega_a(0) = sum_{k>=1} 2^(-mu_a(k)) (order 1: the reference's 6 (1/6 - 0) = 1)
_WALSH_AT_ZERO = {1: 1.0, 2: 1.5, 3: 25 / 18, 4: 407 / 294}


def walsh_part_t(order, delta, t):
    """Torch restatement of the device Walsh part (csrc/fgp_common.h walsh_omega; order 1:
    fast_gp_digital_net_b2.py:297-298) for the generic autograd path (kernel(), derivative-free)."""
    delta = delta.to(torch.int64)
    if order == 1:
        return 6 * (1 / 6 - 2 ** (torch.log2(delta.to(torch.float64)).floor() - t - 1))
    nz = delta != 0
    fl = torch.floor(torch.log2(torch.clamp(delta, min=1).to(torch.float64)))
    beta = t - fl
    x = delta.to(torch.float64) * 2.0 ** (-t)
    t1 = 2.0 ** (-beta)
    if order == 2:
        v = -beta * x + 2.5 * (1 - t1) - 1
    elif order == 3:
        v = beta * x * x - 5 * (1 - t1) * x + 43 / 18 * (1 - t1 * t1) - 1
    else:
        c = 2.0 ** (-(t + 1))
        e1 = torch.full_like(x, 2 * c)
        e2 = torch.full_like(x, 4 / 3 * c * c)
        e3 = torch.full_like(x, 8 / 21 * c ** 3)
        E = torch.zeros_like(x)
        for a in range(t - 1, -1, -1):
            s = 1.0 - 2.0 * ((delta >> (t - 1 - a)) & 1).to(torch.float64)
            E = torch.where(a < beta, E + 0.5 * s * e3, E)
            y = s * 2.0 ** (-(a + 1))
            e3 = e3 + y * e2
            e2 = e2 + y * e1
            e1 = e1 + y
        v = e1 + e2 + e3 + E
    return torch.where(nz, v, torch.full_like(v, _WALSH_AT_ZERO[order]))


_BERN = {
    2: [1.0, -1.0, 1 / 6], 4: [1.0, -2.0, 1.0, 0.0, -1 / 30], 6: [1.0, -3.0, 5 / 2, 0.0, -1 / 2, 0.0, 1 / 42],
    8: [1.0, -4.0, 14 / 3, 0.0, -7 / 3, 0.0, 2 / 3, 0.0, -1 / 30],
}


def _bern(order, x):
    y = 0.0
    for c in _BERN[order]:
        y = y * x + c
    return y


def _bern_t(order, x):
    c = _BERN[order]
    y = torch.zeros_like(x) + c[0]
    for ci in c[1:]:
        y = y * x + ci
    return y
