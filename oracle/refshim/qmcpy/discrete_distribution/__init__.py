"""qmcpy.discrete_distribution stand-in (test infrastructure only; see qmcpy/__init__.py)."""
import numpy as np


class AbstractDiscreteDistribution(object):
    def __init__(self, dimension, replications, seed, d_limit, n_limit):
        self.d = int(dimension) if np.isscalar(dimension) else len(dimension)
        self.replications = 1 if replications is None else replications
        self.seed = seed
        self.d_limit = d_limit
        self.n_limit = n_limit

    def __call__(self, n=None, n_min=None, n_max=None, return_binary=False, warn=True):
        if n is not None:
            n_min, n_max = 0, n
        if n_min is None:
            n_min = 0
        return self._gen_samples(n_min, n_max, False, return_binary, warn)[0]

    def _gen_samples(self, n_min, n_max, return_unrandomized, return_binary, warn):
        raise NotImplementedError


DiscreteDistribution = AbstractDiscreteDistribution
