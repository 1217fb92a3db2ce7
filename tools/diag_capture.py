"""Which part of the C4 bench step cannot be captured into a hipGraph: each phase (reset, fit, post_mean,
post_var) captured on its own after two eager steps, in a fresh process per phase so an invalidated capture does
not poison the next one.  One line per phase: ok / the exception.

    python tools/diag_capture.py            (driver: one subprocess per phase)
    python tools/diag_capture.py PHASE      (one phase)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(phase):
    import torch
    torch.set_default_dtype(torch.float64)
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, 5, 2 ** 20, [1000 + s for s in range(8)], dev)
    g = torch.Generator().manual_seed(3)
    xm = torch.rand((256, 5), generator=g).to(dev)
    xv = torch.rand((8, 5), generator=g).to(dev)

    class A:
        fit_iters = 50
    for _ in range(2):
        bench.step_batched(sh, A, xm, xv)
    torch.cuda.synchronize()
    fns = {"reset": lambda: sh.reset(),
           "fit": lambda: sh.batch.fit(iterations=50, stop_crit_wait_iterations=51),
           "post_mean": lambda: sh.batch.post_mean(xm),
           "post_var": lambda: sh.batch.post_var(xv),
           "step": lambda: bench.step_batched(sh, A, xm, xv)}
    if phase in ("post_mean", "post_var", "fit"):
        sh.reset()
        if phase != "fit":
            sh.batch.fit(iterations=50, stop_crit_wait_iterations=51)
            if phase == "post_var":
                sh.batch.post_mean(xm)
        torch.cuda.synchronize()
    s = torch.cuda.Stream()
    gr = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s, capture_error_mode="thread_local"):
                fns[phase]()
        print("%s: capture ok" % phase, flush=True)
    except Exception as e:
        import traceback
        tb = traceback.format_exc().splitlines()
        print("%s: %s" % (phase, repr(e)[:300]), flush=True)
        for ln in tb[-14:]:
            print("    " + ln, flush=True)


def main():
    if len(sys.argv) > 1:
        one(sys.argv[1])
        return
    for ph in ("reset", "fit", "post_mean", "post_var", "step"):
        r = subprocess.run([sys.executable, "-u", __file__, ph], capture_output=True, text=True, timeout=120)
        print(r.stdout.strip() or ("%s: rc %d %s" % (ph, r.returncode, r.stderr.strip()[-400:])), flush=True)


if __name__ == "__main__":
    main()
