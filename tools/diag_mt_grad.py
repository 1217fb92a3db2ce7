"""GPU diagnostic: the multitask MLL gradient w.r.t. the packed lams from fgp_mt_selinv + fgp_mt_mll_grad
against dense torch autograd of the same blocks (tests/golden fixtures)."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
torch.set_default_dtype(torch.float64)
from golden_util import load_golden
from test_gpu_multitask import product_mt
from fastgaussianprocesses_amd import ops
from fastgaussianprocesses_amd.multitask import _Layout

for name in sys.argv[1:] or ["mt_lattice_d1_a2_T3", "deriv_lattice_d2_a2"]:
    g = load_golden(name)
    gp = product_mt(g)
    lo = _Layout(gp._ns)
    with torch.no_grad():
        packed, gshape = gp._lams_blocks(lo)
    lp = packed.reshape(1, lo.L).detach().clone().requires_grad_(True)
    Y = lo.pack([gp.get_ytilde(l).to(torch.complex128) for l in range(gp.num_tasks)]).reshape(1, -1)
    norm, ld = ops.mt_mll_terms(lo.lay, lp, Y)
    loss = 0.5 * (norm.sum() + ld.sum())
    g1, = torch.autograd.grad(loss, lp)
    # dense
    lp2 = packed.reshape(1, lo.L).detach().clone().requires_grad_(True)
    pos, rows, cols, jj = lo.dense_index(lp2.device)
    M = torch.zeros((1, lo.nmin, lo.R, lo.R), dtype=torch.complex128, device=lp2.device)
    vals = lp2[:, pos]
    M = M.index_put((torch.zeros_like(pos)[None, :], jj[None, :], rows[None, :], cols[None, :]), vals)
    off = rows != cols
    M = M + torch.zeros_like(M).index_put((torch.zeros_like(pos)[None, off], jj[None, off], cols[None, off],
                                            rows[None, off]), vals[:, off].conj())
    A = torch.linalg.inv(M)
    v = Y.reshape(1, lo.R, lo.nmin).permute(0, 2, 1)[..., None]           # [1, nmin, R, 1]
    z = (A @ v)
    n2 = (v.conj() * z).real.sum()
    l2 = 0.5 * (n2 + torch.linalg.slogdet(M).logabsdet.sum())
    g2, = torch.autograd.grad(l2, lp2)
    print(name, "loss", loss.item(), l2.item())
    diag = torch.zeros(lo.L, dtype=torch.bool)
    for k in range(lo.T):
        diag[lo.off[k, k]:lo.off[k, k] + lo.nsrt[k]] = True
    d = (g1 - g2)[0].cpu()
    print("  max |g| dense", float(g2.abs().max()), " diff diag re", float(d[diag].real.abs().max()),
          "diag im", float(d[diag].imag.abs().max()), " off", float(d[~diag].abs().max()) if (~diag).any() else 0)
    with torch.no_grad():
        fac, _, _ = ops.mt_factor(lo.lay, packed.reshape(1, lo.L))
        Z = ops.mt_selinv(lo.lay, fac)[0].cpu()
        Ad = A[0].cpu()                                                       # [nmin, R, R]
        ze = torch.stack([Ad[jj[i], rows[i], cols[i]] for i in range(len(pos))])
        print("  selinv vs dense inverse on the pattern:", float((Z[pos.cpu()] - ze).abs().max()), "scale",
              float(ze.abs().max()))

# end-to-end: d loss / d raw_scale by autograd, by finite differences, and by the chain through the
# packed lams
for name in sys.argv[1:] or ["mt_lattice_d1_a2_T3", "deriv_lattice_d2_a2"]:
    g = load_golden(name)
    gp = product_mt(g)

    def L():
        norm, logdet = gp._norm_logdet()
        return 0.5 * (norm.sum() + logdet.sum())
    loss = L()
    ga, = torch.autograd.grad(loss, gp.raw_scale)
    h = 1e-6
    with torch.no_grad():
        gp.raw_scale.add_(h)
    gp._cache = {}
    lp_ = L().item()
    with torch.no_grad():
        gp.raw_scale.sub_(2 * h)
    gp._cache = {}
    lm_ = L().item()
    with torch.no_grad():
        gp.raw_scale.add_(h)
    gp._cache = {}
    lo = _Layout(gp._ns)
    packed, gshape = gp._lams_blocks(lo)
    gpk, = torch.autograd.grad(packed.real.sum() + packed.imag.sum(), gp.raw_scale)
    print(name, "autograd", ga.tolist(), "fd", (lp_ - lm_) / (2 * h), " d(sum lams)/draw", gpk.tolist(),
          "sum lams - noise", float(packed.real.sum() + packed.imag.sum()))
    # chain: dL/draw = sum Re(conj(dL/dlp) * dlp/draw), dlp/draw = lp - nugget on the diagonal entries
    gp._cache = {}
    lo = _Layout(gp._ns)
    packed, gshape = gp._lams_blocks(lo)
    lpl = packed.reshape(1, lo.L).detach().clone().requires_grad_(True)
    Y = lo.pack([gp.get_ytilde(l).to(torch.complex128) for l in range(gp.num_tasks)]).reshape(1, -1)
    norm, ld = ops.mt_mll_terms(lo.lay, lpl, Y)
    glp, = torch.autograd.grad(0.5 * (norm.sum() + ld.sum()), lpl)
    sig = packed.detach().reshape(-1).clone()
    for k in range(lo.T):
        sig[lo.off[k, k]:lo.off[k, k] + lo.nsrt[k]] -= float(gp.noise)
    print("   chain", float((glp.reshape(-1).conj() * sig).real.sum()))
    # same chain through autograd of packed (retain the graph)
    gch, = torch.autograd.grad(packed.reshape(1, lo.L), gp.raw_scale, grad_outputs=glp)
    print("   autograd chain packed->raw_scale with that upstream", gch.tolist())

    # per pair: VJP of lams[k, l] -> raw_scale with the upstream segment, autograd vs manual
    for (k, l) in lo.pairs:
        a, b = lo.active[k], lo.active[l]
        seg = glp.reshape(-1)[lo.off[k, l]:lo.off[k, l] + lo.nsrt[k]]
        gp._cache = {}
        lam = gp.get_lam(a, b, lo.nsrt[k]) if a <= b else gp.get_lam(b, a, lo.nsrt[k]).conj()
        lam = lam.to(torch.complex128)
        va, = torch.autograd.grad(lam, gp.raw_scale, grad_outputs=seg)
        vm = float((seg.conj() * lam.detach()).real.sum())
        k1 = gp._kernel_from_parts(gp.get_k1parts(min(a, b), max(a, b), lo.nsrt[k]), gp.derivatives[min(a, b)],
                                   gp.derivatives[max(a, b)], gp.derivatives_coeffs[min(a, b)],
                                   gp.derivatives_coeffs[max(a, b)])
        up = seg if a <= b else seg.conj()
        gk = ops.ifftbr_raw(up, True, real_out=True)                # adjoint of ft, real part
        vk = float((gk * k1.detach()).sum())
        print("   pair", (k, l), "tasks", (a, b), "autograd", va.tolist(), "manual", vm, "via ifftbr adjoint", vk,
              "imag k1?", k1.is_complex())
