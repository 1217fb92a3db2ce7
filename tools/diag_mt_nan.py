"""Where the generic multitask autograd loop (FGP_MT_FUSED=0) first produces a non-finite value on the
probnum25-paper-like DSI net (f, grad f) GP (d = 2, alpha = 4, n = 2^10 per task): per iteration the loss,
the raw parameters and their gradients, then the autograd anomaly report of the first bad backward.
(The reference and the device-resident multitask fit stay finite on it: tests/golden/deriv_net_d2_a4_equal_n1024.)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
torch.set_default_dtype(torch.float64)
os.environ["FGP_MT_FUSED"] = "0"


def main():
    from test_gpu_multitask import _paper_gp
    gp = _paper_gp("net", 2, 3, 2 ** 10)
    opt = gp.get_default_optimizer(None)
    mll_const = 3 * 2 ** 10 * 1.8378770664093453
    for it in range(6):
        gp._cache = {k: v for k, v in gp._cache.items() if not k[2]}
        norm, logdet = gp._norm_logdet()
        loss = 0.5 * (norm.sum() + logdet.sum() + mll_const)
        with torch.autograd.detect_anomaly():
            try:
                loss.backward()
            except RuntimeError as e:
                print("iteration", it, "anomaly:", str(e)[:2000])
                return
        print("iteration", it, "loss", loss.item(), "norm", norm.sum().item(), "logdet", logdet.sum().item(),
              {n: (p.detach().cpu().tolist(), None if p.grad is None else p.grad.cpu().tolist())
               for n, p in gp.named_parameters() if p.requires_grad}, flush=True)
        opt.step()
        opt.zero_grad()


if __name__ == "__main__":
    main()
