"""bench.py's secondary lines outside the BASELINE configs: the probnum25 paper's per-step table (its benchmarks and
small fits) and the multitask / batch_multitask notebooks' fits, device engine against the generic autograd loop."""
import os
import time

import numpy as np
import torch

from .common import f_ackley, _clear_capture_error


# ---------------------------------------------------------------- the probnum25 paper's timing table
# docs/examples/probnum25_paper/benchmarks_accuracy_time.tex:6-10 ("time per optimization step", seconds; the
# paper's hardware is unstated): {benchmark: (SI lattice f, SI lattice (f, grad f), DSI net f, DSI net (f, grad f))}
PAPER_S_PER_STEP = {"Ackley": (5.6e-4, 1.3e-3, 7.7e-4, 1.9e-3), "Branin": (5.3e-4, 2.1e-3, 7.0e-4, 3.4e-3),
                    "Camel": (5.0e-4, 2.2e-3, 6.8e-4, 3.4e-3), "StyTang": (5.2e-4, 2.2e-3, 7.7e-4, 3.4e-3),
                    "Hartmann": (5.1e-4, 8.3e-3, 7.1e-4, 1.6e-2)}


def paper_functions():
    """The paper's benchmark functions (probnum25_paper.ipynb cell 7; the standard test-function
    definitions) as (name, d, f, Baker transform for the lattice's (f, grad f) fit) -- cell 15's `funcs`."""
    def branin(x):
        a, b, c, r, s, t = 1.0, 5.1 / (4 * np.pi ** 2), 5 / np.pi, 6.0, 10.0, 1 / (8 * np.pi)
        x1, x2 = 15 * x[:, 0] - 5, 15 * x[:, 1]
        return a * (x2 - b * x1 ** 2 + c * x1 - r) ** 2 + s * (1 - t) * torch.cos(x1) + s

    def camel(x):
        x1, x2 = 6 * x[:, 0] - 3, 4 * x[:, 1] - 2
        return (4 - 2.1 * x1 ** 2 + x1 ** 4 / 3) * x1 ** 2 + x1 * x2 + (-4 + 4 * x2 ** 2) * x2 ** 2

    def styblinski_tang(x):
        x = 10 * x - 5
        return 0.5 * torch.sum(x ** 4 - 16 * x ** 2 + 5 * x, 1)

    def hartmann(x):
        al = torch.tensor([1.0, 1.2, 3.0, 3.2], device=x.device)
        A = torch.tensor([[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14], [3, 3.5, 1.7, 10, 17, 8],
                          [17, 8, 0.05, 10, 0.1, 14]], device=x.device)
        P = 1e-4 * torch.tensor([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                                 [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]],
                                device=x.device, dtype=torch.float64)
        inner = (A[None] * (x[:, None, :] - P[None]) ** 2).sum(-1)
        return -(2.58 + (al * torch.exp(-inner)).sum(1)) / 1.94

    return [("Ackley", 1, f_ackley, False), ("Branin", 2, branin, True), ("Camel", 2, camel, False),
            ("StyTang", 2, styblinski_tang, False), ("Hartmann", 6, hartmann, True)]


def f_grad_f(f, x):
    """(f, df/dx_1, ..., df/dx_d) at x [n, d] -> [n, 1 + d] (probnum25_paper.ipynb cell 7)."""
    xs = [x[:, j].clone().requires_grad_() for j in range(x.shape[1])]
    y = f(torch.stack(xs, 1))
    grads = torch.autograd.grad(y, xs, grad_outputs=torch.ones_like(y))
    return torch.stack([y] + list(grads), 1).detach()


def paper_configs(F, device, log2n=10, iterations=5000, warm=True):
    """The paper's timing protocol (probnum25_paper.ipynb cell 15): n = 2^10 points per task, SI lattice
    alpha = 2 / DSI digital net alpha = 4, f alone (derivatives = [0]) and (f, grad f) (1 + d derivative
    tasks), fit() with the reference's defaults (Rprop lr 0.1, early stopping: improvement 5e-2 over 10
    iterations, at most 5000), store_loss_hist; time per optimisation step = fit wall time / iterations.
    With `warm`, a first untimed pass (3 iterations per config) loads every kernel before the timed pass."""
    n = 2 ** log2n
    if warm:
        paper_configs(F, device, log2n, 3, warm=False)
    out = []
    for name, d, f, bake_grad in paper_functions():
        for fam in ("lattice", "net"):
            for grad in (False, True):
                lbetas = [torch.zeros((1, d), dtype=torch.int64)]
                if grad:
                    lbetas += [e[None] for e in torch.eye(d, dtype=torch.int64)]
                T = len(lbetas)
                if fam == "lattice":
                    gp = F.FastGPLattice([F.Lattice(d, seed=7) for _ in range(T)], derivatives=lbetas, alpha=2,
                                         num_tasks=T, device=device)
                else:
                    gp = F.FastGPDigitalNetB2([F.DigitalNetB2(d, seed=7, randomize="DS") for _ in range(T)],
                                              derivatives=lbetas, alpha=4, num_tasks=T, device=device)
                xs = gp.get_x_next(n * torch.ones(T, dtype=torch.int64))
                ff = (lambda x, f=f: f(1 - 2 * torch.abs(x - 0.5))) if (fam == "lattice" and grad and bake_grad) else f
                if grad:
                    gp.add_y_next([f_grad_f(ff, xs[i])[:, i] for i in range(T)])
                else:
                    gp.add_y_next([f(xs[0])])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                data = gp.fit(iterations=iterations, verbose=0, store_loss_hist=True)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                its = max(1, int(data["iterations"]))
                col = (0 if fam == "lattice" else 2) + (1 if grad else 0)
                out.append({"benchmark": name, "d": d, "gp": "SI lattice alpha=2" if fam == "lattice" else
                            "DSI digital net alpha=4", "data": "(f, grad f)" if grad else "f", "tasks": T,
                            "n_per_task": n, "iterations": its, "s_per_step": el / its,
                            "paper_s_per_step": PAPER_S_PER_STEP[name][col],
                            "class": type(gp).__name__})
                del gp
    return out


def multitask_configs(F, device, iterations=40):
    """The reference's default multitask setting (docs/examples/multitask/fgp_lattice.ipynb cells 3-4: d = 1,
    three tasks -- low / high fidelity Ackley and a cosine sum -- at n = [2^6, 2^3, 2^8], the task kernel
    F F^T + diag(v) LEARNED, abstract_gp.py:116-139) and the same at 16x the points, each fitted `iterations`
    Rprop steps (early stopping off) through the device-resident general multitask fit (fgp_mt_fit_run) and
    through the generic autograd loop (FGP_MT_FUSED=0): time per optimisation step = fit wall time /
    iterations."""
    fs = [lambda x: f_ackley(x, c=0), lambda x: f_ackley(x), lambda x: torch.cos(2 * np.pi * x).sum(1)]
    out = []
    for scale in (1, 16):
        ns = [64 * scale, 8 * scale, 256 * scale]
        row = {"workload": "docs/examples/multitask: FastGPLattice d=1, 3 tasks, n=%s, learned task kernel" % ns,
               "iterations": iterations}
        for path in ("device", "generic"):
            old = os.environ.get("FGP_MT_FUSED")
            os.environ["FGP_MT_FUSED"] = "1" if path == "device" else "0"
            try:
                times = []
                for rep in range(2 if path == "device" else 1):       # the first device pass loads the kernels
                    gp = F.FastGPLattice(1, seed_for_seq=7, num_tasks=3, device=device)
                    xs = gp.get_x_next(n=ns)
                    gp.add_y_next([fs[i](xs[i]) for i in range(3)])
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    data = gp.fit(iterations=iterations, verbose=0, stop_crit_wait_iterations=iterations + 1,
                                  store_loss_hist=True)
                    torch.cuda.synchronize()
                    times.append((time.perf_counter() - t0) / max(1, int(data["iterations"])))
                row[path + "_s_per_step"] = min(times)
                row[path + "_final_loss"] = float(-data["loss_hist"][-1])
                if path == "device":
                    row["device_path"] = "general (fgp_mt_fit_run)" if gp._mt_general_ok() and not gp._mt_fused_ok() \
                        else ("k_mt_spec_iter" if gp._mt_fused_ok() else "generic")
            finally:
                if old is None:
                    os.environ.pop("FGP_MT_FUSED", None)
                else:
                    os.environ["FGP_MT_FUSED"] = old
        row["speedup"] = row["generic_s_per_step"] / row["device_s_per_step"]
        out.append(row)
    out += batch_multitask_configs(F, device, iterations)
    return out


def batch_multitask_configs(F, device, iterations):
    """The reference's parameter-batched multitask setting (docs/examples/batch_multitask/fgp_lattice.ipynb
    cells 4-7: d = 6, shape_batch = [2, 3, 4], 5 tasks at n = 2^[6, 5, 4, 3, 2], scale / lengthscales / noise /
    task factor / task noise batched as in cell 6) and the same at 16x the points: 24 eigen-problems per
    optimisation step through the device fit (fgp_mt_fit_run, G = 24) and through the generic autograd loop."""
    d, T, sb = 6, 5, [2, 3, 4]
    consts = torch.arange(24, device=device, dtype=torch.float64).reshape(sb)
    out = []
    for scale in (1, 16):
        ns = [scale * 2 ** k for k in range(T + 1, 1, -1)]
        row = {"workload": "docs/examples/batch_multitask: FastGPLattice d=6, 5 tasks, n=%s, shape_batch=%s, "
                           "batched scale / lengthscales / noise / task kernel" % (ns, sb), "iterations": iterations}
        for path in ("device", "generic"):
            old = os.environ.get("FGP_MT_FUSED")
            os.environ["FGP_MT_FUSED"] = "1" if path == "device" else "0"
            try:
                times = []
                for rep in range(2 if path == "device" else 1):
                    gp = F.FastGPLattice(d, seed_for_seq=7, num_tasks=T, shape_batch=sb, shape_scale=sb + [1],
                                         shape_lengthscales=sb[1:] + [d], shape_noise=sb[2:] + [1],
                                         shape_factor_task_kernel=sb + [T, T], shape_noise_task_kernel=sb[1:] + [T],
                                         device=device)
                    xs = gp.get_x_next(n=torch.tensor(ns))
                    g = torch.Generator(device=device).manual_seed(11)
                    gp.add_y_next([(consts[..., None, None] * xs[l] ** torch.arange(1, d + 1, device=device)).sum(-1)
                                   + torch.randn(sb + [xs[l].shape[0]], generator=g, device=device) / (3 + l)
                                   for l in range(T)])
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    data = gp.fit(iterations=iterations, verbose=0, stop_crit_wait_iterations=iterations + 1,
                                  store_loss_hist=True)
                    torch.cuda.synchronize()
                    times.append((time.perf_counter() - t0) / max(1, int(data["iterations"])))
                row[path + "_s_per_step"] = min(times)
                row[path + "_final_loss"] = float(-data["loss_hist"][-1])
                if path == "device":
                    row["device_path"] = "general, G=%d (fgp_mt_fit_run)" % 24 if gp._mt_general_ok() else "generic"
            finally:
                if old is None:
                    os.environ.pop("FGP_MT_FUSED", None)
                else:
                    os.environ["FGP_MT_FUSED"] = old
        row["speedup"] = row["generic_s_per_step"] / row["device_s_per_step"]
        out.append(row)
    return out
