"""qmcpy.kernel_methods stand-in (test infrastructure only; see qmcpy/__init__.py).

bernoulli_poly(n, x): Bernoulli polynomial B_n(x), coefficients below, evaluated in Horner form.
weighted_walsh_funcs(order, xb, t): order 1 follows fastgps' own inline formula
(fast_gp_digital_net_b2.py:297-298); orders 2-4 return 1 + omega_order, the series
sum_{k>=0} 2^(-mu_order(k)) wal_k (oracle.fgp_oracle.walsh_omega), so that the reference's
`weighted_walsh_funcs(...) - 1` (:300) is omega.  qmcpy's own values are unavailable offline:
parity at this boundary is unpinned.
"""
from fractions import Fraction as _F

import torch

from . import shift_invar_ops
from . import util

# highest degree first
_BERNOULLI_COEFFS = {
    0: [_F(1)],
    1: [_F(1), _F(-1, 2)],
    2: [_F(1), _F(-1), _F(1, 6)],
    3: [_F(1), _F(-3, 2), _F(1, 2), _F(0)],
    4: [_F(1), _F(-2), _F(1), _F(0), _F(-1, 30)],
    5: [_F(1), _F(-5, 2), _F(5, 3), _F(0), _F(-1, 6), _F(0)],
    6: [_F(1), _F(-3), _F(5, 2), _F(0), _F(-1, 2), _F(0), _F(1, 42)],
    7: [_F(1), _F(-7, 2), _F(7, 2), _F(0), _F(-7, 6), _F(0), _F(1, 6), _F(0)],
    8: [_F(1), _F(-4), _F(14, 3), _F(0), _F(-7, 3), _F(0), _F(2, 3), _F(0), _F(-1, 30)],
}


def bernoulli_poly(n, x):
    coeffs = _BERNOULLI_COEFFS[int(n)]
    y = torch.zeros_like(x) + float(coeffs[0])
    for c in coeffs[1:]:
        y = y * x + float(c)
    return y


def weighted_walsh_funcs(order, xb, t):
    if int(order) == 1:
        return 6 * (1 / 6 - 2 ** (torch.log2(xb).floor() - t - 1))
    from oracle.fgp_oracle import walsh_omega
    return 1 + walsh_omega(int(order), xb, int(t))
