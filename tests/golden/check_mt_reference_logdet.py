"""Reproduces the note in tests/test_oracle_multitask.py: the REAL reference's multitask inverse / logdet cache for a
derivative-informed lattice GP (T = 3, d = 2, n = 128 per task) against a dense per-frequency block check, run in the
build container through oracle/refshim (it prints the three logdets, which agree to 1e-10).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/check_mt_reference_logdet.py
"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
import torch, numpy as np
torch.set_default_dtype(torch.float64)
from oracle.refshim.load_reference import import_reference
fg=import_reference(); import qmcpy
from make_golden import LATTICE_Z
d=2;T=3;seed=11
shifts=[np.random.default_rng(seed+l).uniform(size=d) for l in range(T)]
seqs=[qmcpy.Lattice(d,randomize="SHIFT",generating_vector=LATTICE_Z[:d],shift=shifts[l]) for l in range(T)]
derivs=[torch.tensor([0,0]),torch.tensor([1,0]),torch.tensor([0,1])]
fgp=fg.FastGPLattice(seqs,num_tasks=3,derivatives=derivs,alpha=3)
xs=fgp.get_x_next(n=[128,128,128])
f = lambda x: x[:, 1] * torch.sin(x[:, 0]) + x[:, 0] * torch.cos(x[:, 1])
f0 = lambda x: x[:, 1] * torch.cos(x[:, 0]) + torch.cos(x[:, 1])
f1 = lambda x: torch.sin(x[:, 0]) - x[:, 0] * torch.sin(x[:, 1])
fgp.add_y_next([f(xs[0]),f0(xs[1]),f1(xs[2])])
c=fgp.get_inv_log_det_cache()
print("task order", c.task_order)
inv,ld=c()
print("ref logdet", float(ld))
# dense check like FASTGP_DEBUG
n=c.n[c.task_order]
lams=np.empty((3,3),dtype=object)
for l0 in range(3):
    for l1 in range(l0,3):
        to0,to1=c.task_order[l0],c.task_order[l1]
        lam=fgp.get_lam(to0,to1,n[l0]) if to0<=to1 else fgp.get_lam(to1,to0,n[l0]).conj()
        lams[l0,l1]=torch.sqrt(n[l1])*lam
for l in range(3): lams[l,l]=lams[l,l]+fgp.noise
M=torch.zeros((128,3,3),dtype=torch.complex128)
for a in range(3):
    for b in range(a,3):
        M[:,a,b]=lams[a,b].detach()
        if a!=b: M[:,b,a]=lams[a,b].detach().conj()
print("dense logdet", float(torch.linalg.slogdet(M).logabsdet.sum()))
print("diag imag max", float(torch.stack([lams[l,l].imag.abs().max() for l in range(3)]).max()))
# per-frequency: reference recursion pieces
A0=1/lams[0,0].detach()
ldref = torch.log(torch.abs(lams[0,0].detach()))
dense = torch.linalg.slogdet(M).logabsdet
# recompute reference recursion per frequency (equal n => r=1)
L=[[lams[a,b].detach() if b>=a else None for b in range(3)] for a in range(3)]
A=A0[None,None,:]
ld=ldref.clone()
for l in range(1,3):
    B=torch.stack([L[k][l] for k in range(l)],0)  # [l, n]
    T_=(B[None,:,:]*A).sum(-2)   # [l, n]
    Mm=(B.conj()*T_).sum(-2)
    S=L[l][l]-Mm
    ld=ld+torch.log(torch.abs(S))
    P=T_/S; C=P[:,None,:]*T_[None,:,:].conj()+A
    A=torch.cat([torch.cat([C,-P[:,None,:]],1),torch.cat([-P.conj()[None,:,:],(1/S)[None,None,:]],1)],0)
diff=(ld-dense).abs()
i=int(diff.argmax()); print("max per-freq diff",float(diff.max()),"at",i,"ref",float(ld[i]),"dense",float(dense[i]))
print("top diffs", sorted(diff.tolist())[-5:])
print("eigs at i", torch.linalg.eigvalsh(M[i]))
print("S at i", S[i])
