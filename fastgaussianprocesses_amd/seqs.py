"""Low-discrepancy point sets in NATURAL order (the qmcpy.Lattice / qmcpy.DigitalNetB2 roles).

qmcpy (the reference's point-set dependency, pyproject.toml:39) is not available here, so these
generators take EXPLICIT generating vectors / matrices and shifts; any object exposing the same
duck-typed interface (d, order, replications, randomize, __call__(n_min, n_max[, return_binary]);
DigitalNetB2 also `t`) -- including a real qmcpy instance -- is accepted by the GP classes.

Natural order is what fastgps requires (fast_gp_lattice.py:221, fast_gp_digital_net_b2.py:216):
the first 2^m points of the sequence form a lattice / digital net, which is what makes the Gram
matrix circulant (bit-reversed) / dyadic and the fast transforms exact.
"""
import numpy as np

# Rank-1 lattice generating vector usable for n up to 2^20 (odd components).
DEFAULT_LATTICE_Z = [1, 182667, 469891, 498753, 110745, 446247, 250185, 118627, 245333, 283199]

# Sobol' initial direction numbers (degree s, coefficients a, m_1..m_s) for dimensions 2..8.
_SOBOL_INIT = [
    (1, 0, [1]), (2, 1, [1, 3]), (3, 1, [1, 3, 1]), (3, 2, [1, 1, 1]),
    (4, 1, [1, 1, 3, 3]), (4, 4, [1, 3, 5, 13]), (5, 2, [1, 1, 5, 5, 17]),
]


def radical_inverse_b2(i):
    """v(i) = sum_k bit_k(i) 2^(-k-1) as float64 (exact for i < 2^52)."""
    i = np.asarray(i, dtype=np.uint64)
    r = np.zeros(i.shape, dtype=np.uint64)
    for b in range(52):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(51 - b)
    return r.astype(np.float64) * 2.0 ** -52


def sobol_matrices(d, t=32, mmax=32):
    """Generating-matrix columns (t-bit ints, MSB = first binary digit) of the first d Sobol' dims."""
    if d > 1 + len(_SOBOL_INIT):
        raise ValueError("built-in Sobol' matrices cover d <= %d; pass generating_matrices" % (1 + len(_SOBOL_INIT)))
    C = np.zeros((d, mmax), dtype=np.uint64)
    for k in range(mmax):
        C[0, k] = np.uint64(1) << np.uint64(t - 1 - k)
    for j in range(1, d):
        s, a, m = _SOBOL_INIT[j - 1][0], _SOBOL_INIT[j - 1][1], list(_SOBOL_INIT[j - 1][2])
        for k in range(s, mmax):
            v = m[k - s] ^ (m[k - s] << s)
            for q in range(1, s):
                if (a >> (s - 1 - q)) & 1:
                    v ^= m[k - q] << q
            m.append(v)
        for k in range(mmax):
            C[j, k] = np.uint64(m[k]) << np.uint64(t - 1 - k)
    return C


class Lattice(object):
    """Shifted rank-1 lattice, natural order: x_i = ((v(i) z) % 1 + shift) % 1."""

    def __init__(self, dimension=1, seed=None, randomize="SHIFT", order="NATURAL", generating_vector=None,
                 shift=None):
        if order != "NATURAL":
            raise ValueError("only NATURAL order is supported")
        z = list(DEFAULT_LATTICE_Z) if generating_vector is None else list(generating_vector)
        d = int(dimension)
        while len(z) < d:  # Korobov-style extension beyond the tabulated components
            z.append(int((z[-1] * 182667) % (1 << 20)) | 1)
        self.z = np.asarray(z[:d], dtype=np.int64)
        self.d = d
        self.order = order
        self.replications = 1
        self.randomize = str(randomize).upper() if not isinstance(randomize, bool) else ("SHIFT" if randomize else "FALSE")
        if self.randomize == "SHIFT":
            self.shift = np.asarray(shift if shift is not None else np.random.default_rng(seed).uniform(size=d),
                                    dtype=np.float64)
        elif self.randomize == "FALSE":
            self.shift = np.zeros(d)
        else:
            raise ValueError("Lattice randomize must be SHIFT or FALSE")

    def __call__(self, n_min=0, n_max=None, return_binary=False):
        v = radical_inverse_b2(np.arange(n_min, n_max))
        x = np.outer(v, self.z.astype(np.float64)) % 1
        return (x + self.shift[None, :]) % 1


class DigitalNetB2(object):
    """Base-2 digital net, natural order, t-bit integers with a digital (XOR) shift."""

    def __init__(self, dimension=1, seed=None, randomize="DS", order="NATURAL", generating_matrices=None, t=32,
                 shift=None):
        if order != "NATURAL":
            raise ValueError("only NATURAL order is supported")
        d = int(dimension)
        self.t = int(t)
        C = sobol_matrices(d, t=self.t) if generating_matrices is None else np.asarray(generating_matrices)
        self.C = C.astype(np.uint64)[:d]
        self.d = d
        self.order = order
        self.replications = 1
        self.randomize = str(randomize).upper() if not isinstance(randomize, bool) else ("DS" if randomize else "FALSE")
        if self.randomize == "DS":
            sh = shift if shift is not None else np.random.default_rng(seed).integers(0, 2 ** self.t, size=d,
                                                                                      dtype=np.uint64)
            self.shift = np.asarray(sh).astype(np.uint64)
        elif self.randomize == "FALSE":
            self.shift = np.zeros(d, dtype=np.uint64)
        else:
            raise ValueError("DigitalNetB2 randomize must be DS or FALSE")

    def __call__(self, n_min=0, n_max=None, return_binary=False):
        i = np.arange(n_min, n_max, dtype=np.uint64)
        xb = np.zeros((len(i), self.d), dtype=np.uint64)
        for k in range(self.C.shape[1]):
            bit = ((i >> np.uint64(k)) & np.uint64(1)).astype(bool)
            if bit.any():
                xb[bit] ^= self.C[:, k][None, :]
        xb ^= self.shift[None, :]
        if return_binary:
            return xb
        return xb.astype(np.float64) * 2.0 ** (-self.t)
