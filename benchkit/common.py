"""Shared pieces of bench.py's measurement code: the peaks it prices against, the reference's doctest workload, and the
recovery after an invalidated hipGraph capture."""
import numpy as np
import torch

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6           # MI355X FP64 vector/matrix peak (spec)


def f_ackley(x, a=20, b=0.2, c=2 * np.pi, scaling=32.768):
    # the reference's doctest workload (fastgps/fast_gp_lattice.py:14-22)
    x = 2 * scaling * x - scaling
    t1 = a * torch.exp(-b * torch.sqrt(torch.mean(x ** 2, 1)))
    t2 = torch.exp(torch.mean(torch.cos(c * x), 1))
    return -t1 - t2 + a + np.exp(1)


def _clear_capture_error():
    """After an invalidated capture the HIP error is reported by the next launch: take it here (a throwaway
    op whose error is swallowed) so the eager fallback runs clean."""
    for _ in range(3):
        try:
            torch.zeros(1, device="cuda").add_(1)
            torch.cuda.synchronize()
            return
        except Exception:
            continue
