"""fastgaussianprocesses_amd: MI355X-native fast-transform Gaussian processes.

Drop-in for fastgps' FastGPLattice / FastGPDigitalNetB2 hot path (alegresor/FastGaussianProcesses).
All numerics run in hand-written HIP kernels for gfx950 (fastgaussianprocesses_amd/csrc, C-ABI in
include/fgp_hip.h); there is no CPU fallback.
"""
__version__ = "0.1.0"

from . import ops
from .fast_gp import AbstractFastGP, FastGPDigitalNetB2, FastGPLattice
from .batch import GPBatch, fit_batched
from . import distributed
from .distributed import fit_sharded
from .fit_engine import FusedMLL
from .seqs import DigitalNetB2, Lattice

__all__ = ["FastGPLattice", "FastGPDigitalNetB2", "AbstractFastGP", "Lattice", "DigitalNetB2", "FusedMLL", "GPBatch", "fit_batched", "fit_sharded",
           "distributed", "ops"]
