"""qmcpy.kernel_methods.shift_invar_ops stand-in: BERNOULLIPOLYSDICT keys = allowed orders."""
BERNOULLIPOLYSDICT = {k: None for k in range(1, 5)}
