"""Launch only the prediction kernels of the bench workload (for rocprofv3 --pmc passes).

  python tools/predict_kernels.py [--log2n 20] [--d 5] [--shifts 8] [--n-mean 256] [--n-var 8] [--reps 2]

Builds the bench's batched C4 GPs (bench.Shifts), fits nothing (the initial hyper-parameters are as good
as any for counting bytes and instructions), and runs GPBatch.post_mean / post_var `--reps` times
(k_post_mean, k_sum_chunks, k_qf_rows*, k_qf_cols*, k_qf_finish, k_inv_eig), then one C3 digital-net
GP (n = 2^16, d = 3, alpha = 2) post_mean at N = 256 (the Walsh k_post_mean).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--d", type=int, default=5)
    p.add_argument("--shifts", type=int, default=8)
    p.add_argument("--n-mean", type=int, default=256)
    p.add_argument("--n-var", type=int, default=8)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--c5po", type=int, default=512,
                   help="outputs of the C5 per-output GP (n = 2^18, d = 3, shape_scale = [B, 1]) whose post_mean at "
                        "N = --n-mean also runs (0: skip)")
    a = p.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, a.d, 2 ** a.log2n, [1000 + s for s in range(a.shifts)], dev)
    sh.reset()
    g = torch.Generator().manual_seed(3)
    xm = torch.rand((a.n_mean, a.d), generator=g).to(dev)
    xv = torch.rand((a.n_var, a.d), generator=g).to(dev)
    for _ in range(a.reps):
        sh.batch.post_mean(xm)
        sh.batch.post_var(xv)
    net = F.FastGPDigitalNetB2(F.DigitalNetB2(3, seed=7), device=dev)
    x = net.get_x_next(2 ** 16)
    net.add_y_next(bench.f_ackley(x).contiguous())
    xt = torch.rand((256, 3), generator=g).to(dev)
    for _ in range(a.reps):
        net.post_mean(xt)
    if a.c5po:
        # bench.py's C5 per-output case (secondary_configs): k_post_mean<0, 3, 4, 4> over blocks of 4 outputs
        c5 = bench.MultiOutputGP(F, 18, 3, a.c5po, dev, per_output=True)
        c5.reset()
        xc = torch.rand((a.n_mean, 3), generator=g).to(dev)
        with torch.no_grad():
            c5.gp.coeffs
        for _ in range(a.reps):
            c5.gp.post_mean(xc)
    torch.cuda.synchronize()
    print("ran %d x (post_mean N=%d + post_var N=%d) over %d problems, n=2^%d, d=%d; net post_mean n=2^16 N=256; "
          "C5 per-output post_mean (%d outputs)" % (a.reps, a.n_mean, a.n_var, a.shifts, a.log2n, a.d, a.c5po))


if __name__ == "__main__":
    main()
