"""One step of a bench config, host-profiled and marked for a kernel trace.

  python tools/step_trace.py C2|C3|C5|C5po|C5mix|C4          host enqueue vs GPU time + cProfile top
  rocprofv3 --kernel-trace -d DIR -o t -- python3 tools/step_trace.py C2 ; python tools/step_trace.py --trace CSV
                                                               the marked step's kernels, durations, gaps
"""
import cProfile
import csv
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())


def show_trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    rows = rows[marks[-1] + 1:]
    t0 = int(rows[0]["Start_Timestamp"])
    prev = t0
    busy = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        name = r["Kernel_Name"].replace("void ", "").split("(")[0][:70]
        print("%9.1f us  +gap %7.1f  dur %8.1f  grid %8s  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3,
                                                                  r["Grid_Size_X"], name))
        prev = e
    print("step span %.1f us, busy %.1f us, %d kernels" % ((prev - t0) / 1e3, busy / 1e3, len(rows)))


def main():
    if sys.argv[1] == "--trace":
        show_trace(sys.argv[2])
        return
    import torch
    torch.set_default_dtype(torch.float64)
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    cfg = sys.argv[1]

    class A:
        fit_iters, n_mean, n_var = 50, 256, 8
    g = torch.Generator().manual_seed(3)
    d = 5 if cfg == "C4" else 3
    xm = torch.rand((256, d), generator=g).to(dev)
    xv = torch.rand((8, d), generator=g).to(dev)
    if cfg == "C4":
        sh = bench.Shifts(F, 5, 2 ** 20, [1000 + s for s in range(8)], dev)
        step = lambda: bench.step_batched(sh, A, xm, xv)
    else:
        sg = {"C2": lambda: bench.SingleGP(F, "lattice", 16, 3, dev),
              "C3": lambda: bench.SingleGP(F, "net", 16, 3, dev),
              "C5": lambda: bench.MultiOutputGP(F, 18, 3, 512, dev),
              "C5po": lambda: bench.MultiOutputGP(F, 18, 3, 512, dev, per_output=True),
              "C5mix": lambda: bench.MultiOutputGP(F, 18, 3, 512, dev, torch.float32)}[cfg]()
        step = lambda: bench.step_single(sg, A, xm, xv)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    if cfg != "C4":      # host enqueue time of each phase (no syncs between them)
        t = [time.perf_counter()]
        sg.reset()
        t.append(time.perf_counter())
        sg.gp.fit(iterations=50, stop_crit_wait_iterations=51, verbose=0)
        t.append(time.perf_counter())
        with torch.no_grad():
            sg.gp.coeffs
        t.append(time.perf_counter())
        sg.gp.post_mean(xm)
        t.append(time.perf_counter())
        sg.gp.post_var(xv)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        print("host ms: " + ", ".join("%s %.3f" % (k, 1e3 * (t[i + 1] - t[i])) for i, k in enumerate(
            ("reset", "fit", "coeffs", "post_mean", "post_var", "drain"))))
    torch.cuda._sleep(1000)          # the trace marker: the step's kernels follow the last spin kernel
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%s: host enqueue %.3f ms, until GPU done %.3f ms" % (cfg, (t1 - t0) * 1e3, (t2 - t0) * 1e3))
    st = pstats.Stats(pr).stats          # {(file, line, fn): (cc, nc, tottime, cumtime, callers)}
    rows = sorted(st.items(), key=lambda kv: -kv[1][3])[:45]
    print("%9s %9s %6s  %s" % ("cum_us", "self_us", "calls", "function"))
    for (fn, ln, name), (cc, nc, tt, ct, _) in rows:
        print("%9.1f %9.1f %6d  %s:%d(%s)" % (ct * 1e6, tt * 1e6, nc, os.path.basename(fn), ln, name))


if __name__ == "__main__":
    main()
