"""Golden vectors for fit(masks=...) (abstract_gp.py:152-306: only the outputs y[..., *masks] enter the loss; d_out, the
MLL constant and the logdet term count the selected outputs) from the REAL reference, on the inputs of two committed
multi-output fixtures (lattice_m10_d2_a2_b3: 3 outputs, net_m10_d2_a1_b3: 3 outputs; shared hyper-parameters) with
the masks [[0, 2]] and [[1]]:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_masks.py

Writes tests/golden/masks/<fixture>_mask<k>.npz: the mask, the 6-iteration fit's loss / scale / lengthscale
histories, the fitted raw parameters and post_mean at the fixture's test points after the fit.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.refshim.load_reference import import_reference  # noqa: E402

CASES = [("lattice_m10_d2_a2_b3", [[0, 2]]), ("lattice_m10_d2_a2_b3", [[1]]), ("net_m10_d2_a1_b3", [[0, 2]])]
ITS = 6


def main():
    torch.set_default_dtype(torch.float64)
    fg = import_reference()
    import qmcpy
    os.makedirs(os.path.join(HERE, "masks"), exist_ok=True)
    for k, (name, mask) in enumerate(CASES):
        g = dict(np.load(os.path.join(HERE, name + ".npz")))
        d, B = int(g["d"]), int(g["B"])
        if str(g["family"]) == "lattice":
            seq = qmcpy.Lattice(d, randomize="SHIFT", generating_vector=list(g["z"]), shift=g["shift"])
            gp = fg.FastGPLattice(seq, alpha=int(g["alpha"]), shape_batch=[B])
        else:
            seq = qmcpy.DigitalNetB2(d, randomize="DS", generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                                     shift=g["shift"].astype(np.uint64))
            gp = fg.FastGPDigitalNetB2(seq, alpha=int(g["alpha"]), shape_batch=[B])
        x = gp.get_x_next(2 ** int(g["m"]))
        assert np.array_equal(x.numpy(), g["x"])
        gp.add_y_next(torch.from_numpy(g["y"]))
        data = gp.fit(iterations=ITS, store_hists=True, verbose=0, stop_crit_wait_iterations=ITS + 5,
                      masks=torch.tensor(mask))
        xt = torch.from_numpy(g["x_test"])
        out = dict(source=np.array(name), mask=np.array(mask), loss_hist=data["loss_hist"].detach().numpy(),
                   scale_hist=data["scale_hist"].detach().numpy(),
                   lengthscales_hist=data["lengthscales_hist"].detach().numpy(),
                   raw_scale=gp.raw_scale.detach().numpy(), raw_lengthscales=gp.raw_lengthscales.detach().numpy(),
                   pmean=gp.post_mean(xt).detach().numpy())
        fn = os.path.join(HERE, "masks", "%s_mask%d.npz" % (name, k))
        np.savez_compressed(fn, **out)
        print("wrote", fn, out["loss_hist"][:3])


if __name__ == "__main__":
    main()
