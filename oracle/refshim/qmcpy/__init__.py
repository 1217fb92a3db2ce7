"""Minimal stand-in for the third-party `qmcpy` package (TEST INFRASTRUCTURE ONLY).

The reference (fastgps, /root/reference) depends on qmcpy (pyproject.toml:39 `qmcpy >= 1.6.3b0`;
conda_env.yml:149 pins 1.6.2.1), which is not installed in this container and cannot be
fetched.  This stand-in restates only the published algorithms of the symbols fastgps uses
(symbol list: SURVEY.md §2 row 10) so that the *reference's own orchestration* can run here to
produce golden vectors (tests/golden/make_golden.py).  It is never shipped to, imported by, or
executed from the product package.

Restated algorithms (qmcpy's documented definitions):
  * fftbr_torch(x)  = torch.fft.fft(x[..., bitrev_m], norm="ortho")
  * ifftbr_torch(x) = torch.fft.ifft(x, norm="ortho")[..., bitrev_m]
    Both are pinned by the reference's own doubling recursion (util.py:119-126, 173-178 with
    get_omega fast_gp_lattice.py:261-262) and its FASTGP_DEBUG checks.
  * fwht_torch(x)   = orthonormal Walsh-Hadamard transform in Sylvester (natural) order,
    pinned by the same recursion with omega=1 (fast_gp_digital_net_b2.py:264-265).
  * Lattice: rank-1 lattice in NATURAL (radical-inverse) order, x_i = ((v(i) z) % 1 + shift) % 1,
    with an EXPLICIT generating vector z and shift (qmcpy's default vectors are unavailable).
  * DigitalNetB2: base-2 digital net in NATURAL order, t-bit integers
    xb_i = XOR_{k: bit k of i set} C[:, k], then XOR digital shift; x = xb * 2^-t.
  * kernel_methods.bernoulli_poly(n, x): Bernoulli polynomials B_n, Horner form.
  * kernel_methods.weighted_walsh_funcs(order, xb, t): order 1 as fastgps spells it out
    (fast_gp_digital_net_b2.py:297-298); orders 2..4 restated from the Walsh-series definition
    omega_a(x) = sum_{k>=1} 2^(-mu_a(k)) wal_k(x) (kernel_methods/__init__.py; qmcpy's own values are
    unpinned offline, SURVEY §8c, and tests/test_oracle_golden.py checks the restatement against
    the truncated series).
"""
import numpy as np
import torch

from . import discrete_distribution
from . import kernel_methods
from .discrete_distribution import AbstractDiscreteDistribution, DiscreteDistribution

__version__ = "standin-1.6.2.1"


def _bitrev_indices(m):
    n = 1 << m
    idx = np.arange(n, dtype=np.int64)
    rev = np.zeros(n, dtype=np.int64)
    for b in range(m):
        rev |= ((idx >> b) & 1) << (m - 1 - b)
    return rev


def _bitrev_for(n):
    m = int(np.log2(n))
    assert 2 ** m == n, "n must be a power of 2"
    return torch.from_numpy(_bitrev_indices(m))


def fftbr_torch(x):
    n = x.size(-1)
    br = _bitrev_for(n).to(x.device)
    return torch.fft.fft(x[..., br], norm="ortho")


def ifftbr_torch(x):
    n = x.size(-1)
    br = _bitrev_for(n).to(x.device)
    return torch.fft.ifft(x, norm="ortho")[..., br]


def fwht_torch(x):
    n = x.size(-1)
    m = int(np.log2(n))
    assert 2 ** m == n
    y = x.clone()
    shape = y.shape[:-1]
    h = 1
    while h < n:
        y = y.reshape(shape + (n // (2 * h), 2, h))
        a, b = y[..., 0, :], y[..., 1, :]
        y = torch.stack([a + b, a - b], dim=-2).reshape(shape + (n,))
        h *= 2
    return y / np.sqrt(n)


def _radical_inverse_b2(i):
    """v(i) = sum_k bit_k(i) 2^{-k-1}, exact in float64 for i < 2^52."""
    i = np.asarray(i, dtype=np.uint64)
    r = np.zeros(i.shape, dtype=np.uint64)
    for b in range(52):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(51 - b)
    return r.astype(np.float64) * 2.0 ** -52


class Lattice(AbstractDiscreteDistribution):
    """Rank-1 lattice in NATURAL order with an explicit generating vector and shift."""

    def __init__(self, dimension=1, seed=None, randomize="SHIFT", order="NATURAL",
                 generating_vector=None, shift=None, replications=1):
        assert order == "NATURAL"
        assert generating_vector is not None, "stand-in requires an explicit generating_vector"
        z = np.asarray(generating_vector, dtype=np.int64)
        if np.isscalar(dimension):
            assert len(z) >= dimension
            z = z[:dimension]
        self.z = z
        super().__init__(len(z), replications, seed, np.inf, np.inf)
        self.order = order
        self.randomize = randomize.upper() if isinstance(randomize, str) else ("SHIFT" if randomize else "FALSE")
        if self.randomize == "SHIFT":
            if shift is None:
                shift = np.random.default_rng(seed).uniform(size=self.d)
            self.shift = np.asarray(shift, dtype=np.float64)
        else:
            self.shift = np.zeros(self.d)

    def _gen_samples(self, n_min, n_max, return_unrandomized=False, return_binary=False, warn=True):
        v = _radical_inverse_b2(np.arange(n_min, n_max))
        x = np.outer(v, self.z.astype(np.float64)) % 1
        x = (x + self.shift[None, :]) % 1
        return x[None]


class DigitalNetB2(AbstractDiscreteDistribution):
    """Base-2 digital net in NATURAL order, t-bit integer representation, digital shift."""

    def __init__(self, dimension=1, seed=None, randomize="DS", order="NATURAL",
                 generating_matrices=None, t=32, shift=None, replications=1):
        assert order == "NATURAL"
        assert generating_matrices is not None, "stand-in requires explicit generating_matrices"
        C = np.asarray(generating_matrices, dtype=np.uint64)  # [d, m_max] column ints (t bits, MSB first)
        if np.isscalar(dimension):
            C = C[:dimension]
        self.C = C
        self.t = int(t)
        super().__init__(C.shape[0], replications, seed, np.inf, np.inf)
        self.order = order
        self.randomize = randomize.upper() if isinstance(randomize, str) else ("DS" if randomize else "FALSE")
        if self.randomize == "DS":
            if shift is None:
                shift = np.random.default_rng(seed).integers(0, 2 ** self.t, size=self.d, dtype=np.uint64)
            self.shift = np.asarray(shift, dtype=np.uint64)
        else:
            self.shift = np.zeros(self.d, dtype=np.uint64)

    def _gen_samples(self, n_min, n_max, return_unrandomized=False, return_binary=False, warn=True):
        i = np.arange(n_min, n_max, dtype=np.uint64)
        xb = np.zeros((len(i), self.d), dtype=np.uint64)
        for k in range(self.C.shape[1]):
            bit = ((i >> np.uint64(k)) & np.uint64(1)).astype(bool)
            xb[bit] ^= self.C[:, k][None, :]
        xb ^= self.shift[None, :]
        if return_binary:
            return xb[None]
        return (xb.astype(np.float64) * 2.0 ** (-self.t))[None]


class IIDStdUniform(AbstractDiscreteDistribution):
    def __init__(self, dimension=1, seed=None, replications=1):
        super().__init__(dimension, replications, seed, np.inf, np.inf)
        self.rng = np.random.default_rng(seed)

    def _gen_samples(self, n_min, n_max, return_unrandomized=False, return_binary=False, warn=True):
        return self.rng.uniform(size=(1, n_max - n_min, self.d))
