"""CPU ORACLE for the fast-transform GP hot path — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import this module,
and only as the checker / the timed CPU baseline.  The product package
(fastgaussianprocesses_amd) never imports it and has no CPU fallback.

This is a torch-CPU (fp64) restatement of the reference algorithm, following the reference's op
sequence (bit-reversal gather + torch.fft, autograd backward, torch.optim.Rprop) so that it is both
the numerical spec and a faithful CPU baseline.  Each function cites the reference file:line it
restates.  It is pinned against golden vectors produced by the REAL reference
(tests/golden/make_golden.py, tests/test_oracle_golden.py).

Reference: alegresor/FastGaussianProcesses (fastgps 0.0.4.1a), /root/reference/fastgps/*.py.
Third-party arithmetic: qmcpy (pyproject.toml:39, not installed) — transforms restated from their
published definitions and pinned by the reference's doubling recursion (util.py:113-132,173-178).
"""
import math

import numpy as np
import torch

__all__ = [
    "bitrev_indices", "fftbr", "ifftbr", "fwht", "ft_stable", "ift_stable",
    "bernoulli_poly", "lattice_k1parts", "net_k1parts", "lattice_kernel_parts", "net_kernel_parts",
    "kernel_from_parts", "OracleFastGP", "f_ackley",
]

# --------------------------------------------------------------------------------------------
# Transforms (qmcpy.fftbr_torch / ifftbr_torch / fwht_torch; wrappers abstract_fast_gp.py:197-228)
# --------------------------------------------------------------------------------------------


def bitrev_indices(m):
    """Bit-reversal permutation of range(2^m) (index work: bit-exact)."""
    n = 1 << m
    idx = np.arange(n, dtype=np.int64)
    rev = np.zeros(n, dtype=np.int64)
    for b in range(m):
        rev |= ((idx >> b) & 1) << (m - 1 - b)
    return rev


def _m_of(n):
    m = int(round(math.log2(n))) if n > 0 else -1
    assert n == 1 << m, "n must be a power of 2"
    return m


def fftbr(x):
    """y = fft(x[..., bitrev], norm='ortho') (qmcpy.fftbr_torch; used at fast_gp_lattice.py:224)."""
    br = torch.from_numpy(bitrev_indices(_m_of(x.size(-1))))
    return torch.fft.fft(x[..., br], norm="ortho")


def ifftbr(x):
    """y = ifft(x, norm='ortho')[..., bitrev] (qmcpy.ifftbr_torch; fast_gp_lattice.py:225)."""
    br = torch.from_numpy(bitrev_indices(_m_of(x.size(-1))))
    return torch.fft.ifft(x, norm="ortho")[..., br]


def fwht(x):
    """Orthonormal Sylvester-order Walsh-Hadamard (qmcpy.fwht_torch; fast_gp_digital_net_b2.py:226)."""
    n = x.size(-1)
    _m_of(n)
    y = x.clone()
    shape = y.shape[:-1]
    h = 1
    while h < n:
        y = y.reshape(shape + (n // (2 * h), 2, h))
        a, b = y[..., 0, :], y[..., 1, :]
        y = torch.stack([a + b, a - b], dim=-2).reshape(shape + (n,))
        h *= 2
    return y / np.sqrt(n)


def ft_stable(x, unstable):
    """AbstractFastGP.ft (abstract_fast_gp.py:209-212): mean-centre, transform, add mean*sqrt(n) to bin 0."""
    xmean = x.mean(-1)
    y = unstable(x - xmean[..., None])
    y[..., 0] += xmean * np.sqrt(x.size(-1))
    return y


ift_stable = ft_stable  # abstract_fast_gp.py:225-228 is the same wrapper around ift_unstable

# --------------------------------------------------------------------------------------------
# Kernel parts (fast_gp_lattice.py:263-273, fast_gp_digital_net_b2.py:270-301)
# --------------------------------------------------------------------------------------------

_BERNOULLI = {
    1: [1.0, -1 / 2],
    2: [1.0, -1.0, 1 / 6],
    3: [1.0, -3 / 2, 1 / 2, 0.0],
    4: [1.0, -2.0, 1.0, 0.0, -1 / 30],
    5: [1.0, -5 / 2, 5 / 3, 0.0, -1 / 6, 0.0],
    6: [1.0, -3.0, 5 / 2, 0.0, -1 / 2, 0.0, 1 / 42],
    7: [1.0, -7 / 2, 7 / 2, 0.0, -7 / 6, 0.0, 1 / 6, 0.0],
    8: [1.0, -4.0, 14 / 3, 0.0, -7 / 3, 0.0, 2 / 3, 0.0, -1 / 30],
}


def bernoulli_poly(order, x):
    """Bernoulli polynomial B_order(x), Horner form (qmcpy.kernel_methods.bernoulli_poly)."""
    c = _BERNOULLI[int(order)]
    y = torch.zeros_like(x) + c[0]
    for ci in c[1:]:
        y = y * x + ci
    return y


def lattice_coeff(alpha):
    """(-1)^(alpha+1) (2 pi)^(2 alpha) / (2 alpha)!  (fast_gp_lattice.py:272 with beta=kappa=0)."""
    order = torch.tensor(2 * alpha)
    return (-1) ** (alpha + 1) * torch.exp(2 * alpha * np.log(2 * np.pi) - torch.lgamma(order + 1.0)).item()


def lattice_kernel_parts(x, z, alpha):
    """parts[..., j] for delta = (x - z) % 1 (fast_gp_lattice.py:263-273), alpha per dim (list or int)."""
    delta = (x - z) % 1
    d = delta.size(-1)
    alphas = [alpha] * d if np.isscalar(alpha) else list(alpha)
    return torch.stack([lattice_coeff(alphas[j]) * bernoulli_poly(2 * alphas[j], delta[..., j]) for j in range(d)], -1)


def lattice_k1parts(x, alpha):
    """First-column parts vs x_0 (util.py:50-62 -> abstract_fast_gp.py:173-180)."""
    return lattice_kernel_parts(x, x[:1], alpha)


def walsh_omega(order, delta, t):
    """omega_a(delta / 2^t) = sum_{k>=1} 2^(-mu_a(k)) wal_k(x) for Walsh order a in 2..4, the series
    behind qmcpy.kernel_methods.weighted_walsh_funcs(a, delta, t) - 1 (fast_gp_digital_net_b2.py:300).
    qmcpy is absent offline: this restates the series definition (Dick's weight mu_a(k) = sum of the
    a highest bit positions of k, +1 each) by a digit recursion -- y_a = (-1)^(x_{a+1}) 2^-(a+1),
    elementary symmetric sums e_r of the digits above the current one, seeded with the all-zero tail:
        omega = sum_{r<a} e_r(all) + sum_{b < beta} (1/2) s_b e_{a-1}(y_{>b})
    (the k whose lower bits are free sum to 2^b [x_1..x_b = 0]).  It is checked against the
    truncated series itself in tests/test_oracle_golden.py.  PARITY UNPINNED against qmcpy."""
    from math import prod
    delta = torch.as_tensor(delta).to(torch.int64)
    r1 = order - 1
    c = 2.0 ** -(t + 1)
    e = [torch.ones(delta.shape, dtype=torch.float64)]
    for r in range(1, order):
        e.append(torch.full(delta.shape, c ** r * 2.0 ** (-r * (r - 1) / 2) / prod(1 - 2.0 ** -i for i in range(1, r + 1)),
                            dtype=torch.float64))
    nz = delta != 0
    hi = torch.zeros(delta.shape, dtype=torch.int64)          # floor(log2 delta), exact
    for b in range(64):
        hi = torch.where((delta >> b) > 0, torch.full_like(hi, b), hi)
    beta = torch.where(nz, t - hi, torch.full_like(hi, 1 << 30))
    E = torch.zeros(delta.shape, dtype=torch.float64)
    for a in range(t - 1, -1, -1):
        s = 1.0 - 2.0 * ((delta >> (t - 1 - a)) & 1).to(torch.float64)
        E = E + torch.where(a < beta, 0.5 * s * e[r1], torch.zeros_like(E))
        y = s * 2.0 ** -(a + 1)
        for r in range(r1, 0, -1):
            e[r] = e[r] + y * e[r - 1]
    K = 2.0 ** (-r1 * (r1 - 1) / 2) / prod(1 - 2.0 ** -i for i in range(1, r1 + 1))
    tail = 0.5 * K * 2.0 ** (-(t + 2) * r1) / (1 - 2.0 ** -r1)     # b >= t, reached only by delta = 0
    E = E + torch.where(nz, torch.zeros_like(E), torch.full_like(E, tail))
    return sum(e[1:]) + E


def net_kernel_parts(xb, zb, t, alpha=1):
    """Digitally-shift-invariant parts for delta = xb XOR zb (fast_gp_digital_net_b2.py:274-301):
    order 1 by the reference's inline formula (:297-298), orders 2-4 by walsh_omega (:300)."""
    delta = xb ^ zb
    d = delta.shape[-1]
    alphas = [alpha] * d if np.isscalar(alpha) else list(alpha)
    cols = []
    for j in range(d):
        if int(alphas[j]) == 1:
            cols.append(6 * (1 / 6 - 2 ** (torch.log2(delta[..., j]).floor() - t - 1)))
        else:
            cols.append(walsh_omega(int(alphas[j]), delta[..., j], t))
    return torch.stack(cols, -1)


def net_k1parts(xb, t, alpha=1):
    return net_kernel_parts(xb, xb[:1], t, alpha)


def net_to_b(x, t):
    """_convert_to_b (fast_gp_digital_net_b2.py:270-271)."""
    return torch.floor((x % 1) * 2 ** t).to(torch.int64)


def kernel_from_parts(parts, scale, lengthscales):
    """scale * prod_j(1 + l_j parts_j) (abstract_fast_gp.py:181-191, beta=kappa=0, single term)."""
    ndim = parts.ndim
    s = scale.reshape(scale.shape + torch.Size([1] * (ndim - 2)))
    ls = lengthscales.reshape(lengthscales.shape[:-1] + torch.Size([1] * (ndim - 1) + [lengthscales.size(-1)]))
    return (s * (1 + ls * parts).prod(-1))


def f_ackley(x, a=20, b=0.2, c=2 * np.pi, scaling=32.768):
    """The reference's doctest workload (fast_gp_lattice.py:14-22)."""
    x = 2 * scaling * x - scaling
    t1 = a * torch.exp(-b * torch.sqrt(torch.mean(x ** 2, 1)))
    t2 = torch.exp(torch.mean(torch.cos(c * x), 1))
    return -t1 - t2 + a + np.exp(1)


# --------------------------------------------------------------------------------------------
# Single-task fast GP (AbstractGP/AbstractFastGP + util caches, single-task branches)
# --------------------------------------------------------------------------------------------


class OracleFastGP(object):
    """Restatement of FastGPLattice / FastGPDigitalNetB2, single task, beta=kappa=0.

    family: "lattice" (x float points in [0,1)) or "net" (xb int64 t-bit points).
    y: [*shape_batch, n].  scale [...,1], lengthscales [...,d], noise [1] (raw = log, tfs exp).
    """

    def __init__(self, family, x, xb, y, alpha=2, t=None, scale=1.0, lengthscales=1.0, noise=None,
                 shape_scale=(1,), shape_lengthscales=None, requires_grad_noise=False):
        assert torch.get_default_dtype() == torch.float64
        self.family = family
        self.x = x
        self.xb = xb
        self.t = t
        self.alpha = alpha
        self.y = y
        self.n = y.size(-1)
        self.d = x.size(-1)
        self.shape_batch = y.shape[:-1]
        if noise is None:
            noise = 1e-8 if family == "lattice" else 1e-16  # fast_gp_lattice.py:132 / fast_gp_digital_net_b2.py:127
        if shape_lengthscales is None:
            shape_lengthscales = (self.d,)
        # raw parameters through tfs=(log, exp) (fast_gp_lattice.py:137-139, abstract_gp.py:78-111)
        self.raw_scale = torch.nn.Parameter(torch.log(scale * torch.ones(shape_scale)))
        self.raw_lengthscales = torch.nn.Parameter(torch.log(lengthscales * torch.ones(shape_lengthscales)))
        self.raw_noise = torch.nn.Parameter(torch.log(noise * torch.ones(1)), requires_grad=requires_grad_noise)
        self.ft_unstable = fftbr if family == "lattice" else fwht
        self.ift_unstable = ifftbr if family == "lattice" else fwht
        self._k1parts = None
        self._ytilde = None

    # hyperparameters (abstract_gp.py:622-639)
    @property
    def scale(self):
        return torch.exp(self.raw_scale)

    @property
    def lengthscales(self):
        return torch.exp(self.raw_lengthscales)

    @property
    def noise(self):
        return torch.exp(self.raw_noise)

    def parameters(self):
        return [p for p in [self.raw_scale, self.raw_lengthscales, self.raw_noise]]

    def ft(self, v):
        return ft_stable(v, self.ft_unstable)

    def ift(self, v):
        return ft_stable(v, self.ift_unstable)

    def k1parts(self):
        if self._k1parts is None:
            if self.family == "lattice":
                self._k1parts = lattice_k1parts(self.x, self.alpha)
            else:
                self._k1parts = net_k1parts(self.xb, self.t, self.alpha)
        return self._k1parts

    def k1(self):
        return kernel_from_parts(self.k1parts(), self.scale, self.lengthscales)

    def lam(self):
        """_LamCaches (util.py:95-112): lam = ft(k1)."""
        return self.ft(self.k1())

    def ytilde(self):
        """_YtildeCache (util.py:168-172)."""
        if self._ytilde is None:
            if self.n > 1:
                self._ytilde = self.ft(self.y)
            else:
                self._ytilde = self.y.clone().to(torch.complex128 if self.family == "lattice" else torch.float64)
        return self._ytilde

    def inv_logdet(self):
        """_FastInverseLogDetCache.__call__ single-task branch (util.py:277-300)."""
        lams = np.sqrt(self.n) * self.lam() + self.noise
        logdet = torch.log(torch.abs(lams)).sum(-1)
        return 1 / lams, logdet

    def norm_logdet(self):
        """get_norm_term_logdet_term (util.py:364-370, tilde solve util.py:354-363)."""
        A, logdet = self.inv_logdet()
        yt = self.ytilde()
        z = yt * A
        norm = (yt.conj() * z).real.sum(-1, keepdim=True)
        return norm, logdet[..., None]

    def mll_loss(self):
        """MLL loss exactly as fit() assembles it (abstract_gp.py:230,235,253-261)."""
        d_out = int(torch.tensor(self.shape_batch).prod())
        norm, logdet = self.norm_logdet()
        term1 = norm.sum()
        term2 = d_out / torch.tensor(logdet.shape).prod() * logdet.sum()
        return 0.5 * (term1 + term2 + d_out * self.n * np.log(2 * np.pi)), term1, term2

    def gram_solve(self, v):
        """gram_matrix_solve (util.py:338-353), single task: ift(A * ft(v)).real."""
        A, _ = self.inv_logdet()
        return self.ift(self.ft(v) * A).real

    def coeffs(self):
        """_CoeffsCache (util.py:419-425)."""
        return self.gram_solve(self.y)

    def kernel(self, x, z):
        """_kernel (abstract_fast_gp.py:192-196) on float points."""
        if self.family == "lattice":
            parts = lattice_kernel_parts(x, z, self.alpha)
        else:
            parts = net_kernel_parts(net_to_b(x, self.t) if torch.is_floating_point(x) else x,
                                     net_to_b(z, self.t) if torch.is_floating_point(z) else z, self.t, self.alpha)
        return kernel_from_parts(parts, self.scale, self.lengthscales)

    def _train_pts(self):
        return self.x if self.family == "lattice" else self.xb

    def post_mean(self, xt, chunk=64):
        """post_mean (abstract_gp.py:352-380), chunked over test points to bound memory."""
        with torch.no_grad():
            c = self.coeffs()
            outs = []
            for i0 in range(0, xt.size(0), chunk):
                k = self.kernel(xt[i0:i0 + chunk, None, :], self._train_pts()[None, :, :])
                outs.append(torch.einsum("...i,...i->...", k, c[..., None, :]))
            return torch.cat(outs, -1)

    def post_var(self, xt):
        """post_var (abstract_gp.py:381-416), single task, n = self.n."""
        with torch.no_grad():
            kmat_new = self.kernel(xt, xt)
            kmat = self.kernel(xt[:, None, :], self._train_pts()[None, :, :])  # [..., N, n]
            # permute N in front of the batch dims before the solve (abstract_gp.py:409-411)
            t = self.gram_solve(kmat.movedim(-2, 0)).movedim(0, -2)
            diag = kmat_new - (t * kmat).sum(-1)
            diag[diag < 0] = 0
            return diag

    def post_cov(self, x0, x1):
        """post_cov (abstract_gp.py:417-474), single task."""
        with torch.no_grad():
            kmat_new = self.kernel(x0[:, None, :], x1[None, :, :])
            k1 = self.kernel(x0[:, None, :], self._train_pts()[None, :, :])
            k2 = self.kernel(x1[:, None, :], self._train_pts()[None, :, :])
            t = self.gram_solve(k2.movedim(-2, 0)).movedim(0, -2)  # abstract_gp.py:455-457
            return kmat_new - (k1[..., :, None, :] * t[..., None, :, :]).sum(-1)

    def post_cubature_mean(self):
        """abstract_fast_gp.py:65-81 (task kernel == 1)."""
        with torch.no_grad():
            return (self.scale * self.coeffs()).sum(-1)

    def post_cubature_var(self):
        """abstract_fast_gp.py:82-109 (single task: inv[...,0] is 1/ev_0, nsqrts = n)."""
        with torch.no_grad():
            A, _ = self.inv_logdet()
            term = (self.n * A[..., 0]).real
            pcvar = self.scale[..., 0] - self.scale[..., 0] ** 2 * term
            pcvar[pcvar < 0] = 0.
            return pcvar

    def fit(self, iterations=5000, lr=0.1, stop_crit_improvement_threshold=5e-2, stop_crit_wait_iterations=10):
        """AbstractGP.fit, MLL branch (abstract_gp.py:152-306) with the default Rprop(lr=0.1)
        (abstract_fast_gp.py:53-57).  Returns dict with iterations and histories."""
        params = [p for p in self.parameters() if p.requires_grad]
        opt = torch.optim.Rprop(params, lr=lr)
        logtol = np.log(1 + stop_crit_improvement_threshold)
        best = math.inf
        save = math.inf
        wait = 0
        loss_hist, scale_hist, ls_hist = [], [], []
        best_params = None
        for i in range(iterations + 1):
            loss, _, _ = self.mll_loss()
            lv = loss.item()
            if lv < best:
                best = lv
                best_params = [self.raw_scale.data.clone(), self.raw_lengthscales.data.clone(), self.raw_noise.data.clone()]
            if (save - lv) > logtol:
                wait = 0
                save = best
            else:
                wait += 1
            brk = i == iterations or wait == stop_crit_wait_iterations
            loss_hist.append(-lv)
            scale_hist.append(self.scale.detach().clone())
            ls_hist.append(self.lengthscales.detach().clone())
            if brk:
                break
            loss.backward()
            opt.step()
            opt.zero_grad()
        self.raw_scale.data.copy_(best_params[0])
        self.raw_lengthscales.data.copy_(best_params[1])
        self.raw_noise.data.copy_(best_params[2])
        return {"iterations": i, "loss_hist": torch.tensor(loss_hist),
                "scale_hist": torch.stack(scale_hist), "lengthscales_hist": torch.stack(ls_hist)}


# --------------------------------------------------------------------------------------------
# Point sets (qmcpy.Lattice / DigitalNetB2 natural order, explicit generators)
# --------------------------------------------------------------------------------------------


def lattice_points(z, shift, n_min, n_max):
    """x_i = ((v(i) z) % 1 + shift) % 1, v = base-2 radical inverse (natural order)."""
    i = np.arange(n_min, n_max, dtype=np.uint64)
    r = np.zeros(i.shape, dtype=np.uint64)
    for b in range(52):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(51 - b)
    v = r.astype(np.float64) * 2.0 ** -52
    x = np.outer(v, np.asarray(z, dtype=np.float64)) % 1
    return (x + np.asarray(shift)[None, :]) % 1


def net_points_binary(C, shift, n_min, n_max):
    """xb_i = XOR_{k: bit k of i} C[:, k]  XOR shift (natural order, t-bit ints)."""
    C = np.asarray(C).astype(np.uint64)
    i = np.arange(n_min, n_max, dtype=np.uint64)
    xb = np.zeros((len(i), C.shape[0]), dtype=np.uint64)
    for k in range(C.shape[1]):
        bit = ((i >> np.uint64(k)) & np.uint64(1)).astype(bool)
        xb[bit] ^= C[:, k][None, :]
    xb ^= np.asarray(shift).astype(np.uint64)[None, :]
    return xb.astype(np.int64)
