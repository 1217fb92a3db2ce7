"""Where the time of the spectral fit iteration goes (C4 shape: 8 shifted lattice GPs, n = 2^20, d = 5):
device-clock stamps of every workgroup (start, each wave's end) over `--iters` launches of the fused
k_spec_tile (the step's own launch: streaming + partials + the two-level reduction + Rprop) and of the
stage launch (streaming + partials only), reported as offsets from the launch's first workgroup start:
start spread, workgroup durations, end-time percentiles, and the tail = last end - the end of the
last workgroup that does no reduction work.  One JSON line per variant; FGP_LIB_PATH selects an
experiment build (tools/build_exp.sh).

    python tools/exp_spec_stamps.py [--iters 20] [--log2n 20] [--d 5] [--shifts 8]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def placement(st, grid):
    """FGP_EXP_HWID builds (tools/build_exp.sh): the start stamp's bits 48-63 hold the workgroup's XCC and
    se / sh / cu ids -> per launch, how many workgroups shared each CU, and the mean workgroup duration by that
    count (is the spread of the durations the CUs' uneven loading?)"""
    ids = (st[:, :grid, 0] >> 48)
    if not bool((ids != 0).any()):
        return None
    clk = st[:, :grid].clone()
    clk[:, :, 0] &= (1 << 48) - 1
    dur = (clk[:, :, 1:].amax(2) - clk[:, :, 0]).double()
    by = {}
    for i in range(st.shape[0]):
        row = ids[i].tolist()
        cnt = {}
        for v in row:
            cnt[v] = cnt.get(v, 0) + 1
        for w, v in enumerate(row):
            by.setdefault(cnt[v], []).append(float(dur[i, w]))
    # the workgroups sharing a CU, by start order (the older one wins the SIMDs' issue arbitration), and by XCD
    first, second, xcd = [], [], {}
    for i in range(st.shape[0]):
        grp = {}
        for w, v in enumerate(ids[i].tolist()):
            grp.setdefault(v, []).append(w)
            xcd.setdefault(v >> 8, []).append(float(dur[i, w]))
        for v, ws in grp.items():
            if len(ws) == 2:
                a, b = sorted(ws, key=lambda w: int(clk[i, w, 0]))
                first.append(float(dur[i, a]))
                second.append(float(dur[i, b]))
    mean = lambda v: sum(v) / max(1, len(v))
    return {"cus_used_per_launch": float(sum(len(set(ids[i].tolist())) for i in range(st.shape[0])) / st.shape[0]),
            "wg_dur_ticks_by_wgs_per_cu": {k: (len(v), sum(v) / len(v)) for k, v in sorted(by.items())},
            "dur_ticks_first_started_on_cu": mean(first), "dur_ticks_second_started_on_cu": mean(second),
            "frac_second_longer": mean([1.0 if b > a else 0.0 for a, b in zip(first, second)]),
            "dur_ticks_by_xcd": {k: round(mean(v), 1) for k, v in sorted(xcd.items())}}


def summarize(st, grid, khz, name, extra=None):
    """st [iters, grid, 5] raw wall-clock stamps -> offsets in us"""
    pl = placement(st, grid)
    st = st[:, :grid].clone()
    st[:, :, 0] &= (1 << 48) - 1
    st = st.double()
    t0 = st[:, :, 0].amin(1, keepdim=True)
    start = (st[:, :, 0] - t0) * (1e3 / khz)
    end = (st[:, :, 1:].amax(2) - t0) * (1e3 / khz)
    dur = end - start
    se, _ = end.sort(1)
    q = lambda x, p: float(x.quantile(p))
    out = {"variant": name, "grid": grid, "launches": st.shape[0],
           "span_us": float(se[:, -1].mean()),
           "start_p50_us": q(start, 0.5), "start_p99_us": q(start, 0.99), "start_max_us": float(start.amax(1).mean()),
           "dur_p10_us": q(dur, 0.1), "dur_p50_us": q(dur, 0.5), "dur_p90_us": q(dur, 0.9),
           "end_p50_us": q(end, 0.5), "end_p90_us": q(end, 0.9),
           # the 17 latest workgroups include the 16 level-1 group finishers and the level-2 finisher
           "end_18th_latest_us": float(se[:, -18].mean()), "end_2nd_latest_us": float(se[:, -2].mean())}
    out["tail_us"] = out["span_us"] - out["end_18th_latest_us"]
    if pl is not None:
        out["placement"] = pl
    if extra:
        out.update(extra)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--d", type=int, default=5)
    ap.add_argument("--shifts", type=int, default=8)
    args = ap.parse_args()
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    n = 2 ** args.log2n
    sh = bench.Shifts(F, args.d, n, bench.shard_seeds(0, 1, args.shifts), dev)
    sh.reset()
    eng = F.batch.batched_engine(sh.gps, args.iters + 4)
    eng.run(0, 2)
    torch.cuda.synchronize()
    assert eng.basis is not None, "the spectral path is not selected"
    grid = bench.spec_tile_grid(n, eng.d, eng.G)
    khz = bench.wall_clock_khz(F, dev)
    it = args.iters
    stamps = torch.zeros((it, max(grid, 1), 5), dtype=torch.int64, device=dev)
    # fused launches (the step's own: fgp_fit_run, one iteration each)
    torch.cuda._sleep(int(2.4e9 * 2e-4 * it))
    for i in range(it):
        eng._nll.stamps = stamps[i].data_ptr()
        eng.run(i, 1)
    eng._nll.stamps = None
    torch.cuda.synchronize()
    print(json.dumps(summarize(stamps.cpu(), grid, khz, "fused k_spec_tile")), flush=True)
    # events around one enqueue of all iterations (the step's form)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2.4e9 * 2e-4))
    a.record()
    eng.run(0, it)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"variant": "fused fgp_fit_run, events", "us_per_iter": 1e3 * a.elapsed_time(b) / it}),
          flush=True)
    # stage launches (streaming + partials, no reduction)
    stamps.zero_()
    torch.cuda._sleep(int(2.4e9 * 2e-4 * it))
    for i in range(it):
        eng._nll.stamps = stamps[i].data_ptr()
        eng.stage(0)
    eng._nll.stamps = None
    torch.cuda.synchronize()
    print(json.dumps(summarize(stamps.cpu(), grid, khz, "stage k_spec_tile")), flush=True)
    a.record()
    for i in range(it):
        eng.stage(0)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"variant": "stage launches, events", "us_per_iter": 1e3 * a.elapsed_time(b) / it}), flush=True)
    # streaming calibration: a plain read of the spectra + Y (torch sum)
    bas = eng.basis
    ys = eng.ysq
    for _ in range(2):
        bas.sum()
    a.record()
    for _ in range(10):
        bas.sum()
        ys.sum()
    b.record()
    torch.cuda.synchronize()
    us = 1e3 * a.elapsed_time(b) / 10
    mb = (bas.numel() + ys.numel()) * 8 / 1e6
    print(json.dumps({"variant": "torch sum of spectra + Y", "us": us, "MB": mb, "GBps": mb * 1e3 / us}), flush=True)


if __name__ == "__main__":
    main()
