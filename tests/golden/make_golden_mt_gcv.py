"""Golden vectors for fit(loss_metric="GCV" / "CV") of multitask GPs with equal n per task and a fixed task kernel (the
derivative-informed setting: util.py:371-394 with T tasks, abstract_gp.py:242-272) from the REAL reference, on the
inputs of the committed fixtures deriv_net_d2_a4_equal / deriv_lattice_d2_a2_equal (make_golden_multitask.py):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mt_gcv.py [--metric GCV|CV]

Writes tests/golden/mt_gcv/<fixture>.npz (GCV) or tests/golden/mt_cv/<fixture>.npz (CV): the 6-iteration fit's loss /
scale / lengthscale histories, the fitted raw parameters and post_mean at the fixture's test points after the fit.  (A lattice fixture is skipped if the
reference's complex-valued lattice GCV makes its fit raise, as it does for one task.)
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.refshim.load_reference import import_reference  # noqa: E402

NAMES = ["deriv_net_d2_a4_equal", "deriv_lattice_d2_a2_equal"]
ITS = 6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--metric", default="GCV", choices=["GCV", "CV"])
    metric = ap.parse_args().metric
    sub = "mt_gcv" if metric == "GCV" else "mt_cv"
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    os.makedirs(os.path.join(HERE, sub), exist_ok=True)
    for name in NAMES:
        g = dict(np.load(os.path.join(HERE, name + ".npz")))
        d, ns = int(g["d"]), [int(v) for v in g["ns"]]
        T = len(ns)
        kw = dict(alpha=int(g["alpha"]), num_tasks=T, derivatives=[torch.from_numpy(v) for v in g["derivatives"]])
        if str(g["family"]) == "lattice":
            seqs = [qmcpy.Lattice(d, randomize="SHIFT", generating_vector=list(g["z"]), shift=g["shifts"][l])
                    for l in range(T)]
            gp = fg.FastGPLattice(seqs, **kw)
        else:
            seqs = [qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                                       shift=g["shifts"][l].astype(np.uint64)) for l in range(T)]
            gp = fg.FastGPDigitalNetB2(seqs, **kw)
        xs = gp.get_x_next(n=ns)
        for l in range(T):
            assert np.array_equal(xs[l].numpy(), g["x_%d" % l])
        gp.add_y_next([torch.from_numpy(g["y_%d" % l]) for l in range(T)])
        try:
            data = gp.fit(loss_metric=metric, iterations=ITS, store_hists=True, verbose=0,
                          stop_crit_wait_iterations=ITS + 5)
        except TypeError as e:
            print("skip", name, "(the reference's fit raised: %s)" % e)
            continue
        xt = torch.from_numpy(g["x_test"])
        out = dict(source=np.array(name), loss_hist=data["loss_hist"].detach().numpy(),
                   scale_hist=data["scale_hist"].detach().numpy(),
                   lengthscales_hist=data["lengthscales_hist"].detach().numpy(),
                   raw_scale=gp.raw_scale.detach().numpy(), raw_lengthscales=gp.raw_lengthscales.detach().numpy(),
                   pmean=gp.post_mean(xt).detach().numpy())
        fn = os.path.join(HERE, sub, name + ".npz")
        np.savez_compressed(fn, **out)
        print("wrote", fn, out["loss_hist"][:3])


if __name__ == "__main__":
    main()
