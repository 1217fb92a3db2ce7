"""qmcpy.kernel_methods.util stand-in."""
from .. import shift_invar_ops
