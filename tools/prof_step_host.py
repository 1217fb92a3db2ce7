"""Where the eager time of a small bench step goes (C2 / C3: n = 2^16, d = 3; VERDICT r05 "What's weak" #3 / #4).

For bench.SingleGP + bench.step_single's fit: HIP-event time of the eager `reset + fit` (what the bench's phases_ms
report as ytilde+fit), its host wall time, the same sequence replayed from a hipGraph, and a cProfile of the eager
host work (the fixed costs around the single-launch fit).

    python tools/prof_step_host.py [--family lattice|net] [--reps 20]
"""
import argparse
import cProfile
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="lattice")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--detail", action="store_true", help="also print the callees of the fit's host functions")
    ap.add_argument("--segments", action="store_true",
                    help="host time of each piece of the eager fit, called one by one (no profiler overhead)")
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sg = bench.SingleGP(F, args.family, 16, 3, dev)
    its = dict(iterations=args.iters, stop_crit_wait_iterations=args.iters + 1, verbose=0)

    def one():
        sg.reset()
        sg.gp.fit(**its)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    ev = []
    walls = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        one()
        e1.record()
        walls.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1))
    from fastgaussianprocesses_amd import fit_engine as E
    gu0 = E.persist_giveups()
    g, info = bench.capture_fn(lambda: (one(), sg.gp.raw_lengthscales.detach())[1:])
    gms = None
    if g is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        gms = e0.elapsed_time(e1) / args.reps
    # the same replays one at a time with an idle host gap before each (the eager sequence leaves the GPU idle
    # while the host prepares the next launches): device time per replay
    gap = []
    if g is not None:
        for _ in range(args.reps):
            torch.cuda.synchronize()
            time.sleep(0.002)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            gap.append(e0.elapsed_time(e1))
        gap.sort()
    gu1 = E.persist_giveups()
    ev.sort()
    walls.sort()
    print(json.dumps({"family": args.family, "eager_events_ms_median": ev[len(ev) // 2],
                      "eager_host_ms_median": 1e3 * walls[len(walls) // 2], "graph_ms": gms, "graph_after_idle_ms_median": gap[len(gap) // 2] if gap else None,
                      "graph_info": info, "persist_giveups_during_replays": gu1 - gu0}), flush=True)
    if args.segments:
        segments(sg, args)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    for _ in range(5):
        one()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr).stats
    rows = sorted(st.items(), key=lambda kv: -kv[1][3])[:70]
    print("%9s %9s %6s  %s" % ("cum_us/5", "self_us/5", "calls", "function"))
    for (fn, ln, name), (cc, nc, tt, ct, _) in rows:
        print("%9.1f %9.1f %6d  %s:%d(%s)" % (ct * 2e5, tt * 2e5, nc, os.path.basename(fn), ln, name))
    if args.detail:
        ps = pstats.Stats(pr)
        for fn in ("_fused_engine", "_spec_basis", "_ysq", "cached_engine", "refill", "reset", "add_y_next",
                   "_restore_best", "run_persist", "persist_result", "_parts_gen", "spec_basis_gen", "fit"):
            ps.print_callees(r"\b%s\b" % fn)


def segments(sg, args):
    """Median host microseconds of the pieces FastGP.fit runs before / after the single-launch fit's launch, each
    called on its own (the device drained before each rep, so a piece's time is its host work + launch calls)."""
    import math
    gp = sg.gp
    rows = {}

    def t(name, fn):
        t0 = time.perf_counter()
        r = fn()
        rows.setdefault(name, []).append(1e6 * (time.perf_counter() - t0))
        return r
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t("reset (bench)", sg.reset)
        n = gp._nh
        t("fit checks (_fused_ok)", gp._fused_ok)
        t("spectra (_spec_basis)", lambda: gp._spec_basis(n, 1))
        t("ytilde (get_ytilde)", gp.get_ytilde)
        t("Y (_ysq)", lambda: gp._ysq(None, 1))
        eng = t("engine (_fused_engine, inputs cached)", lambda: gp._fused_engine(args.iters, 0.1))
        t("persist launch (run_persist)", lambda: eng.run_persist(args.iters, math.log(1.05), args.iters + 1, defer=True))
        t("restore best (_restore_best)", lambda: gp._restore_best(eng, eng.raw))
        t("control word (persist_result, waits)", eng.persist_result)
        eng.release_inputs()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sg.reset()
        gp.fit(iterations=args.iters, stop_crit_wait_iterations=args.iters + 1, verbose=0)
        rows.setdefault("whole reset + fit (host, until return)", []).append(1e6 * (time.perf_counter() - t0))
    for k, v in rows.items():
        v.sort()
        print("%-44s %8.1f us" % (k, v[len(v) // 2]), flush=True)


if __name__ == "__main__":
    main()
