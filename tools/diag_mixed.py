"""Measure the mixed-precision (data_dtype=float32) multi-output path against the fp64 CPU oracle on
the same fp32-rounded observations (C5 shape, reduced outputs): loss trajectory, fitted parameters,
posterior mean / variance errors, at two nuggets.   python tools/diag_mixed.py [--m 18] [--B 16]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.set_default_dtype(torch.float64)
import fastgaussianprocesses_amd as F  # noqa: E402
from oracle import fgp_oracle as O  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=18)
    p.add_argument("--B", type=int, default=16)
    p.add_argument("--its", type=int, default=5)
    a = p.parse_args()
    n, d, B = 2 ** a.m, 3, a.B
    for noise in (1e-8, 1e-3):
        res = {}
        for dt in (torch.float64, torch.float32):
            gp = F.FastGPLattice(F.Lattice(d, seed=7), shape_batch=[B], noise=noise, device="cuda", data_dtype=dt)
            x = gp.get_x_next(n).cpu()
            f = O.f_ackley(x)
            g = torch.Generator().manual_seed(5)
            y = torch.stack([f * (1 + b / B) + 0.01 * torch.randn(f.shape, generator=g) for b in range(B)])
            y32 = y.float().double()
            gp.add_y_next(y32.to("cuda"))
            data = gp.fit(iterations=a.its, store_loss_hist=True, verbose=0, stop_crit_wait_iterations=a.its + 5)
            xt = torch.rand((64, d), generator=torch.Generator().manual_seed(17))
            pm = gp.post_mean(xt.to("cuda")).cpu()
            pv = gp.post_var(xt[:4].to("cuda")).cpu()
            res[dt] = (data["loss_hist"], gp.raw_lengthscales.detach().cpu(), pm, pv)
        o = O.OracleFastGP("lattice", x, None, y32, alpha=2, noise=noise)
        od = o.fit(iterations=a.its, stop_crit_wait_iterations=a.its + 5)
        opm = o.post_mean(xt)
        opv = o.post_var(xt[:4])
        kxx = float(o.kernel(xt[:4], xt[:4]).abs().max())
        for dt, (lh, ls, pm, pv) in res.items():
            print("noise %.0e %s: loss rel %.3e  ls abs %.3e  pmean rel %.3e  pvar/kxx %.3e" % (
                noise, str(dt).split(".")[-1], float((lh - od["loss_hist"]).abs().max() / od["loss_hist"].abs().max()),
                float((ls - o.raw_lengthscales.detach()).abs().max()), float((pm - opm).abs().max() / opm.abs().max()),
                float((pv - opv).abs().max()) / kxx))


if __name__ == "__main__":
    main()
