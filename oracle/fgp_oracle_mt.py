"""CPU ORACLE for MULTITASK and DERIVATIVE-INFORMED fast GPs — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only tests/ may import this module (as the checker).  The product package never imports it.

A torch-CPU (fp64) restatement of the reference's num_tasks > 1 / derivatives paths.  The block
inverse is stated DIFFERENTLY from the reference on purpose: the reference inverts the T x T block
matrix of eigenvalue vectors by a recursive Schur-complement bordering (util.py:299-323); here the
transform-domain Gram matrix is written out as n_min independent dense R x R Hermitian blocks, one per
frequency class j (R = sum_k n_k / n_min), and each is inverted with torch.linalg (inv / slogdet).  The
two agree to rounding, and the golden fixtures made by the REAL reference
(tests/golden/make_golden_multitask.py) pin this statement (tests/test_oracle_golden.py).

Frequency-class structure (derivation of the reference's reshapes, util.py:303-320, 356-360): with
tasks sorted by n descending (util.py:273), task k's transformed vector of length n_k is laid out as
n_k / n_min rows of n_min; the Gram block between tasks k <= l (n_k >= n_l) is diagonal in the sense
  Lambda[(k, q), (l, p)](j) = lams[k, l][q n_min + j]   iff  p == q mod (n_l / n_min)
(q, p rows of the two tasks, j < n_min the frequency class), and zero otherwise; lams[k, l] =
sqrt(n_l) lam_{k,l} (n_k-point transform of the cross first column, util.py:284-285), the nugget is on
the diagonal blocks (util.py:286-293) and everything is multiplied by the task kernel (util.py:294-298).

Reference: alegresor/FastGaussianProcesses (fastgps 0.0.4.1a), /root/reference/fastgps/*.py.
"""
import math

import numpy as np
import torch

from .fgp_oracle import (bernoulli_poly, fftbr, ifftbr, fwht, ft_stable, walsh_omega, lattice_points,
                         net_points_binary)

__all__ = ["lattice_parts_deriv", "net_parts_deriv", "kernel_from_parts_deriv", "OracleMultiTaskFastGP"]


def lattice_parts_deriv(delta, beta, kappa, alpha):
    """FastGPLattice._kernel_parts_from_delta (fast_gp_lattice.py:267-273): order 2 alpha - beta - kappa,
    coefficient (-1)^(alpha + kappa + 1) (2 pi)^(2 alpha) / order!  (alpha, beta, kappa per dimension)."""
    alpha = torch.as_tensor(alpha, dtype=torch.int64)
    order = 2 * alpha - beta - kappa
    assert (order >= 2).all(), "order must all be at least 2"
    coeff = (-1) ** (alpha + kappa + 1) * torch.exp(2 * alpha * np.log(2 * np.pi) - torch.lgamma(order + 1.0))
    return coeff * torch.stack([bernoulli_poly(int(order[j]), delta[..., j]) for j in range(delta.size(-1))], -1)


def net_parts_deriv(delta, beta, kappa, alpha, t):
    """FastGPDigitalNetB2._kernel_parts_from_delta (fast_gp_digital_net_b2.py:289-301):
    (-2)^(beta + kappa) (ind + omega_{alpha - beta - kappa}(delta)), ind = [beta + kappa > 0]."""
    alpha = torch.as_tensor(alpha, dtype=torch.int64)
    bpk = beta + kappa
    ind = (bpk > 0).to(torch.int64)
    order = alpha - bpk
    assert (order >= 1).all() and (order <= 4).all()
    cols = []
    for j in range(delta.size(-1)):
        o = int(order[j])
        if o == 1:
            cols.append(6 * (1 / 6 - 2 ** (torch.log2(delta[..., j].to(torch.float64)).floor() - t - 1)))
        else:
            cols.append(walsh_omega(o, delta[..., j], t))
    omega = torch.stack(cols, -1)
    return (-2) ** bpk * (ind + omega)


def kernel_from_parts_deriv(parts, scale, lengthscales, beta0, beta1, c0, c1):
    """_kernel_from_parts (abstract_fast_gp.py:181-191): parts [..., p0, p1, d]."""
    ndim = parts.ndim
    s = scale.reshape(scale.shape + torch.Size([1] * (ndim - 2)))
    ls = lengthscales.reshape(lengthscales.shape[:-1] + torch.Size([1] * (ndim - 1) + [lengthscales.size(-1)]))
    ind = ((beta0[:, None, :] + beta1[None, :, :]) == 0).to(torch.int64)
    terms = s * (ind + ls * parts).prod(-1)
    return ((terms * c1).sum(-1) * c0).sum(-1)


class OracleMultiTaskFastGP(object):
    """num_tasks >= 1 fast GP with optional derivative multi-indices per task.

    family "lattice" (explicit z + per-task shift) or "net" (explicit generating matrices C, t, per-task
    digital shift).  ys[l]: [*shape_batch, n_l].  Default hyper-parameters as the reference
    (fast_gp_lattice.py:129-158, abstract_gp.py:58-150)."""

    def __init__(self, family, gen, shifts, ys, alpha=2, t=32, derivatives=None, derivatives_coeffs=None,
                 noise=None, adaptive_nugget=False):
        self.family, self.gen, self.shifts, self.alpha, self.t = family, gen, shifts, alpha, t
        self.T = len(ys)
        self.ys = ys
        self.ns = [int(y.size(-1)) for y in ys]
        self.d = len(shifts[0])
        self.shape_batch = ys[0].shape[:-1]
        self.adaptive_nugget = adaptive_nugget
        T, d = self.T, self.d
        deriv = derivatives is not None or derivatives_coeffs is not None
        if derivatives is None:
            derivatives = [torch.zeros((1, d), dtype=torch.int64) for _ in range(T)]
        self.derivatives = [b[None, :] if b.ndim == 1 else b for b in derivatives]
        if derivatives_coeffs is None:
            derivatives_coeffs = [torch.ones(len(b)) for b in self.derivatives]
        self.coeffs_d = derivatives_coeffs
        if noise is None:
            noise = 1e-8 if family == "lattice" else 1e-16
        self.raw_scale = torch.nn.Parameter(torch.zeros(1))
        self.raw_lengthscales = torch.nn.Parameter(torch.zeros(d))
        self.raw_noise = torch.nn.Parameter(torch.log(noise * torch.ones(1)), requires_grad=False)
        rank = 1 if (deriv or T > 1) else 0
        self.raw_factor_task_kernel = torch.nn.Parameter(torch.ones((T, rank)), requires_grad=(T > 1 and not deriv))
        if deriv:
            self._ntk_tf = lambda v: v                       # identity tfs, value 0 (abstract_gp.py:59-62)
            self.raw_noise_task_kernel = torch.nn.Parameter(torch.zeros(T), requires_grad=False)
        else:
            self._ntk_tf = torch.exp
            self.raw_noise_task_kernel = torch.nn.Parameter(torch.zeros(T), requires_grad=T > 1)
        self._pts = [None] * T

    # hyper-parameters
    @property
    def scale(self):
        return torch.exp(self.raw_scale)

    @property
    def lengthscales(self):
        return torch.exp(self.raw_lengthscales)

    @property
    def noise(self):
        return torch.exp(self.raw_noise)

    @property
    def gram_matrix_tasks(self):
        """F F^T + diag(noise_task_kernel) (util.py:157-162)."""
        F = self.raw_factor_task_kernel
        return F @ F.T + self._ntk_tf(self.raw_noise_task_kernel)[..., None] * torch.eye(self.T)

    def parameters(self):
        return [self.raw_scale, self.raw_lengthscales, self.raw_noise, self.raw_factor_task_kernel,
                self.raw_noise_task_kernel]

    # points (explicit generators)
    def points(self, l, n):
        """first n points of task l: (float points, kernel-argument points)."""
        if self.family == "lattice":
            x = torch.from_numpy(lattice_points(self.gen, self.shifts[l], 0, n))
            return x, x
        xb = torch.from_numpy(net_points_binary(self.gen, self.shifts[l], 0, n))
        return xb.to(torch.float64) * 2.0 ** (-self.t), xb

    def to_b(self, x):
        return torch.floor((x % 1) * 2 ** self.t).to(torch.int64)

    # transforms
    def ft(self, v):
        return ft_stable(v, fftbr if self.family == "lattice" else fwht)

    def ift(self, v):
        return ft_stable(v, ifftbr if self.family == "lattice" else fwht)

    # kernel
    def parts(self, xa, zb, beta0, beta1):
        """_kernel_parts (abstract_fast_gp.py:173-180): [..., p0, p1, d]."""
        if self.family == "lattice":
            delta = (xa - zb) % 1
        else:
            delta = xa ^ zb
        out = torch.empty(tuple(delta.shape[:-1]) + (len(beta0), len(beta1), self.d))
        for a in range(len(beta0)):
            for b in range(len(beta1)):
                if self.family == "lattice":
                    out[..., a, b, :] = lattice_parts_deriv(delta, beta0[a], beta1[b], [self.alpha] * self.d)
                else:
                    out[..., a, b, :] = net_parts_deriv(delta, beta0[a], beta1[b], [self.alpha] * self.d, self.t)
        return out

    def kernel(self, x, z, ta, tb):
        if self.family == "net":
            x = self.to_b(x) if torch.is_floating_point(x) else x
            z = self.to_b(z) if torch.is_floating_point(z) else z
        p = self.parts(x, z, self.derivatives[ta], self.derivatives[tb])
        return kernel_from_parts_deriv(p, self.scale, self.lengthscales, self.derivatives[ta], self.derivatives[tb],
                                       self.coeffs_d[ta], self.coeffs_d[tb])

    def k1parts(self, a, b, n):
        """_K1PartsSeq[a, b][:n] (util.py:50-62): points of task a vs the first point of task b."""
        _, pa = self.points(a, n)
        _, pb = self.points(b, 1)
        return self.parts(pa, pb[0], self.derivatives[a], self.derivatives[b])

    def lam(self, a, b, n):
        """_LamCaches[a, b][log2 n] (util.py:95-112): ft of the first-column kernel (a <= b)."""
        k1 = kernel_from_parts_deriv(self.k1parts(a, b, n), self.scale, self.lengthscales, self.derivatives[a],
                                     self.derivatives[b], self.coeffs_d[a], self.coeffs_d[b])
        return self.ft(k1)

    def ytilde(self, l):
        """_YtildeCache (util.py:168-172)."""
        y = self.ys[l]
        if self.ns[l] > 1:
            return self.ft(y)
        return y.clone().to(torch.complex128 if self.family == "lattice" else torch.float64)

    # transform-domain Gram blocks
    def order(self, ns):
        return torch.tensor(ns).argsort(descending=True)     # util.py:273 (same call, same order)

    def blocks(self, ns):
        """Dense per-frequency-class blocks Lam [R, R, n_min] (complex) in sorted task order."""
        to = self.order(ns).tolist()
        nsrt = [ns[i] for i in to]
        act = [k for k in range(self.T) if nsrt[k] > 0]
        nmin = min(nsrt[k] for k in act)
        R = sum(nsrt[k] // nmin for k in act)
        rs = [sum(nsrt[kk] // nmin for kk in act[:i]) for i in range(len(act))]
        Kt = self.gram_matrix_tasks
        lams = {}
        for i, k in enumerate(act):
            for l in act[i:]:
                a, b = to[k], to[l]
                lam = self.lam(a, b, nsrt[k]) if a <= b else self.lam(b, a, nsrt[k]).conj()
                lams[k, l] = math.sqrt(nsrt[l]) * lam.to(torch.complex128)
        if self.adaptive_nugget:
            tr00 = lams[to.index(0), to.index(0)].sum(-1)
            for k in act:
                lams[k, k] = lams[k, k] + self.noise * (lams[k, k].sum(-1) / tr00).abs()
        else:
            for k in act:
                lams[k, k] = lams[k, k] + self.noise
        for (k, l) in list(lams):
            lams[k, l] = lams[k, l] * Kt[to[k], to[l]]
        Lam = torch.zeros((R, R, nmin), dtype=torch.complex128)
        for i, k in enumerate(act):
            for ii, l in enumerate(act):
                if l < k:
                    continue
                v = lams[k, l].reshape(-1, nmin)               # [n_k / n_min, n_min]
                for q in range(nsrt[k] // nmin):
                    p = q % (nsrt[l] // nmin)
                    Lam[rs[i] + q, rs[ii] + p] = v[q]
                    if l != k:
                        Lam[rs[ii] + p, rs[i] + q] = v[q].conj()
        return Lam, to, nsrt, nmin, R

    def inv_logdet(self, ns=None):
        ns = self.ns if ns is None else ns
        Lam, to, nsrt, nmin, R = self.blocks(ns)
        M = Lam.permute(2, 0, 1)                               # [n_min, R, R]
        A = torch.linalg.inv(M).permute(1, 2, 0)               # [R, R, n_min]
        logdet = torch.linalg.slogdet(M).logabsdet.sum()
        return A, logdet, to, nsrt, nmin

    def _apply(self, A, zs, to, nmin):
        """_gram_matrix_solve_tilde_to_tilde (util.py:354-363): per-task transformed vectors -> A z."""
        zc = torch.cat([zs[o].to(torch.complex128) for o in to], -1)
        zc = zc.reshape(zc.shape[:-1] + (-1, nmin))             # [..., R, n_min]
        out = torch.einsum("rcj,...cj->...rj", A, zc).reshape(zc.shape[:-2] + (-1,))
        parts = out.split([self.ns_for_split[o] for o in to], -1)
        res = [None] * self.T
        for i, o in enumerate(to):
            res[o] = parts[i]
        return res

    def norm_logdet(self):
        """get_norm_term_logdet_term (util.py:364-370)."""
        A, logdet, to, nsrt, nmin = self.inv_logdet()
        self.ns_for_split = self.ns
        yts = [self.ytilde(l) for l in range(self.T)]
        zs = self._apply(A, yts, to, nmin)
        norm = sum((yts[l].conj() * zs[l]).real.sum(-1, keepdim=True) for l in range(self.T))
        return norm, logdet

    def mll_loss(self):
        d_out = int(torch.tensor(self.shape_batch).prod())
        norm, logdet = self.norm_logdet()
        return 0.5 * (norm.sum() + d_out * logdet + d_out * sum(self.ns) * np.log(2 * np.pi))

    def gram_solve(self, v, ns=None):
        """gram_matrix_solve (util.py:338-353): v [..., sum n] in task order."""
        ns = self.ns if ns is None else list(ns)
        A, _, to, nsrt, nmin = self.inv_logdet(ns)
        self.ns_for_split = ns
        vs = v.split(ns, -1)
        vts = [self.ft(vs[l]) for l in range(self.T)]
        zs = self._apply(A, vts, to, nmin)
        return torch.cat([self.ift(zs[l]).real for l in range(self.T)], -1)

    def coeffs(self):
        return self.gram_solve(torch.cat(self.ys, -1))

    # predictions (abstract_gp.py:352-474, abstract_fast_gp.py:65-154)
    def _kmat(self, x, tasks, ns):
        Kt = self.gram_matrix_tasks
        rows = []
        for t in tasks:
            rows.append(torch.cat([Kt[t, l] * self.kernel(x[:, None, :], self.points(l, ns[l])[1][None, :, :], t, l)
                                   for l in range(self.T)], -1))
        return torch.stack(rows, 0)                              # [T', N, sum n]

    def post_mean(self, x):
        with torch.no_grad():
            kmat = self._kmat(x, range(self.T), self.ns)
            return torch.einsum("tni,...i->...tn", kmat, self.coeffs())

    def post_var(self, x, ns=None):
        with torch.no_grad():
            ns = self.ns if ns is None else list(ns)
            Kt = self.gram_matrix_tasks
            knew = torch.stack([Kt[t, t] * self.kernel(x, x, t, t) for t in range(self.T)], 0)
            kmat = self._kmat(x, range(self.T), ns)
            tt = self.gram_solve(kmat, ns)
            diag = knew - (tt * kmat).sum(-1)
            diag[diag < 0] = 0
            return diag

    def post_cov(self, x0, x1):
        with torch.no_grad():
            Kt = self.gram_matrix_tasks
            T = self.T
            knew = torch.stack([torch.stack([Kt[a, b] * self.kernel(x0[:, None, :], x1[None, :, :], a, b)
                                             for b in range(T)], 0) for a in range(T)], 0)
            k1 = self._kmat(x0, range(T), self.ns)
            k2 = self._kmat(x1, range(T), self.ns)
            tt = self.gram_solve(k2)
            return knew - torch.einsum("ani,bmi->abnm", k1, tt)

    def post_cubature_mean(self):
        with torch.no_grad():
            Kt = self.gram_matrix_tasks
            cs = self.coeffs().split(self.ns, -1)
            return torch.stack([sum((self.scale * cs[l]).sum(-1) * Kt[t, l] for l in range(self.T))
                                for t in range(self.T)], -1)

    def _cub_term(self, ns):
        A, _, to, nsrt, nmin = self.inv_logdet(ns)
        nord = torch.tensor(nsrt, dtype=torch.float64)
        mvec = torch.cat([torch.zeros(1), (nord / nord[-1]).cumsum(0)]).to(torch.int64)[:-1]
        nsq = torch.sqrt(nord[:, None] * nord[None, :])
        cut = A[mvec][:, mvec][..., 0]
        Kt = self.gram_matrix_tasks.to(torch.complex128)
        return Kt[:, to], nsq * cut, Kt[to, :]

    def post_cubature_var(self, ns=None):
        with torch.no_grad():
            ns = self.ns if ns is None else list(ns)
            left, mid, right = self._cub_term(ns)
            term = torch.einsum("ij,jk,ki->i", left, mid, right).real
            Kt = self.gram_matrix_tasks
            pcvar = self.scale * torch.diagonal(Kt) - self.scale ** 2 * term
            pcvar[pcvar < 0] = 0.
            return pcvar

    def post_cubature_cov(self):
        with torch.no_grad():
            left, mid, right = self._cub_term(self.ns)
            term = torch.einsum("ij,jk,kl->il", left, mid, right).real
            cov = self.scale * self.gram_matrix_tasks - self.scale ** 2 * term
            dg = torch.diagonal(cov)
            dg[dg < 0] = 0.
            return cov

    def fit(self, iterations=3, lr=0.1, stop_crit_improvement_threshold=5e-2, stop_crit_wait_iterations=10):
        """AbstractGP.fit MLL branch (abstract_gp.py:152-306), Rprop(lr=0.1) over every parameter."""
        opt = torch.optim.Rprop(self.parameters(), lr=lr)
        logtol = np.log(1 + stop_crit_improvement_threshold)
        best, save, wait, best_params = math.inf, math.inf, 0, None
        hist = {"loss_hist": [], "scale_hist": [], "lengthscales_hist": [], "task_kernel_hist": []}
        for i in range(iterations + 1):
            loss = self.mll_loss()
            lv = loss.item()
            if lv < best:
                best = lv
                best_params = [p.data.clone() for p in self.parameters()]
            if (save - lv) > logtol:
                wait, save = 0, best
            else:
                wait += 1
            brk = i == iterations or wait == stop_crit_wait_iterations
            hist["loss_hist"].append(-lv)
            hist["scale_hist"].append(self.scale.detach().clone())
            hist["lengthscales_hist"].append(self.lengthscales.detach().clone())
            hist["task_kernel_hist"].append(self.gram_matrix_tasks.detach().clone())
            if brk:
                break
            loss.backward()
            opt.step()
            opt.zero_grad()
        for p, v in zip(self.parameters(), best_params):
            p.data.copy_(v)
        out = {k: torch.stack(v) if k != "loss_hist" else torch.tensor(v) for k, v in hist.items()}
        out["iterations"] = i
        return out
