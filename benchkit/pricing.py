"""bench.py's pricing of the measured kernels: the fit kernels' geometry and algorithmic bytes, their live device-clock /
HIP-event timing, and the rooflines read from the rocprofv3 kernel-trace and PMC summaries committed under profiles/
(the dominant kernel of the headline line and of every secondary line)."""
import json
import os

import torch

from .common import FP64_PEAK_TFS, HBM_PEAK_GBS, _clear_capture_error


STAGES = ("k_fwd_rows", "k_fwd_cols", "k_bwd_rows")
SPEC_BLOCKS = 512      # k blocks per problem of the spectral iteration (csrc/fgp_nll.h kSpecBlocks)


SPEC_RING, SPEC_LDS_MAX, SPEC_MAX_DMA = 2, 80 * 1024, 6      # csrc/fgp_nll.h kSpecRing / kSpecLdsMax / kSpecMaxDma


def stage_names(variant):
    """The fit-iteration kernels of a variant, in launch order (the reduce + Rprop step aside; the fused
    spectral kernel includes it)."""
    if variant == "spectral_fused":
        return ("k_spec_tile",)
    return ("k_spec_iter",) if variant == "spectral" else STAGES


def spec_tile_geometry(n, d, G, shared=True, family=0):
    """(workgroups, problems per wave, problem groups) of the LDS-ring tile kernel k_spec_tile, or None when
    spec_geometry picks the per-wave k_spec_iter (the conditions of csrc/fgp_spectral.hip spec_geometry)."""
    main = n // 2 if family == 0 else n
    nb = min(SPEC_BLOCKS, max(1, main // 64))
    if not (shared and d <= 5 and main >= 256) or os.environ.get("FGP_SPEC_TILE", "1")[:1] == "0":
        return None
    ppw = 2 if G >= 2 else 1
    pg = (G + ppw - 1) // ppw
    pgp = 1 if pg <= 1 else (2 if pg <= 2 else 4)
    ck = 64 * (4 // pgp)
    rows = 2 ** d + G
    ok = (pg <= 4 and rows * ck * 8 * SPEC_RING <= SPEC_LDS_MAX and rows * ck <= 512 * SPEC_MAX_DMA and
          (rows * ck) % 128 == 0 and rows * ck >= 256 and nb % (4 // pgp) == 0 and main % (64 * nb) == 0)
    if ok:
        return (nb // (4 // pgp), ppw, pg)
    # problem slices (G > 8): PS = 4 PPW problems per workgroup, one k block each (64 chunks per workgroup,
    # more blocks while the grid has < 512 workgroups), snb x slices workgroups
    sppw = 4 if d <= 3 else 2
    ps = 4 * sppw
    srows = 2 ** d + ps
    nsl = (G + ps - 1) // ps
    snb = max(1, main // (64 * 64))
    while snb * nsl < 512 and snb * 2 <= max(1, main // 64):
        snb *= 2
    snb = min(snb, nb)
    if (pg > 4 and srows * 64 * 8 * SPEC_RING <= SPEC_LDS_MAX and srows * 64 <= 512 * SPEC_MAX_DMA and
            (srows * 64) % 128 == 0 and main % (64 * snb) == 0):
        return (snb * nsl, sppw, 4)
    return None


def spec_geometry(n, d, G, shared=True, family=0):
    """(k blocks, problems per wave, problem groups) of the spectral iteration (csrc/fgp_spectral.hip
    spec_geometry): the tile kernel's when it applies, else k_spec_iter's."""
    main = n // 2 if family == 0 else n
    nb = min(SPEC_BLOCKS, max(1, main // 64))
    t = spec_tile_geometry(n, d, G, shared, family)
    if t is not None:
        ps = 4 * t[1]
        sliced = (G + t[1] - 1) // t[1] > 4          # problem slices: the grid is k blocks x slices
        return (t[0] // ((G + ps - 1) // ps) if sliced else nb), t[1], t[2]
    ppw = 2 if (G >= 2 and shared and d <= 5) else 1
    if ppw == 2 and G > 8 and d <= 3:
        ppw = 4
    return nb, ppw, (G + ppw - 1) // ppw


def spec_tile_grid(n, d, G, shared=True, family=0):
    """Workgroups of the LDS-ring tile kernel k_spec_tile, or None (per-wave k_spec_iter)."""
    t = spec_tile_geometry(n, d, G, shared, family)
    return None if t is None else t[0]


def spec_fused(n, d, G):
    """fgp_fit_run runs the whole iteration (streaming + reduction + Rprop) as ONE k_spec_tile launch:
    tile geometry, per-problem parameters, G <= 8 (csrc/fgp_nll.hip fgp_fit_run)."""
    return spec_tile_grid(n, d, G) is not None and G <= 8


def r2c_active(n):
    """The lattice fit runs the half-length (R2C) or real-even (RE) kernels for n >= 2^17 unless
    FGP_R2C=0 (csrc/fgp_nll.hip to_nll)."""
    return n >= 2 ** 17 and os.environ.get("FGP_R2C", "2")[:1] != "0"


def fit_variant(n, parts_array):
    """'re' (real-even kernels: n >= 2^17 with regenerated parts, the default), 'r2c' (FGP_R2C=1, or a
    parts array) or 'full' (n < 2^17 or FGP_R2C=0) -- the choice of csrc/fgp_nll.hip to_nll."""
    if not r2c_active(n):
        return "full"
    if parts_array or os.environ.get("FGP_R2C", "2")[:1] == "1":
        return "r2c"
    return "re"


def re_row_log2():
    """Row length log2 of the real-even kernels' n/2-point transform (csrc/fgp_nll_re.hip kP2reDefault)."""
    return 11


def fit_grid(n, P, variant, d=5):
    """{stage kernel: (workgroups per fit launch, threads per workgroup)}."""
    if variant == "spectral_fused":
        return {"k_spec_tile": (spec_tile_grid(n, d, P), 256)}
    if variant == "spectral":
        if spec_tile_grid(n, d, P) is not None:       # staged tile launches (problem slices when P > 8)
            return {"k_spec_tile": (spec_tile_grid(n, d, P), 256)}
        nb, _, pg = spec_geometry(n, d, P)
        return {"k_spec_iter": ((nb * pg + 3) // 4, 256)}
    if variant == "re":     # N1 = n / (2 N2) rows of N2: N1/2 row-pair workgroups of N2/8, n/16384 column tiles
        N2 = 2 ** re_row_log2()
        N1 = n // (2 * N2)
        return {"k_fwd_rows": (P * N1 // 2, N2 // 8), "k_fwd_cols": (P * n // 16384, 256),
                "k_bwd_rows": (P * N1 // 2, N2 // 8)}
    g = P * max(1, (n // 2 if variant == "r2c" else n) // 4096)
    return {k: (g, 256) for k in STAGES}


def stage_bytes(n, d, P, parts_array, variant=None):
    """Algorithmic (compulsory) HBM bytes of one launch of each fit-iteration kernel over P lattice
    problems (complex128 intermediate `work` of L complex values; float64 Y; DESIGN.md 'Kernels'):
      full (L = n):  rows 16L write (+ 8nd parts), cols 16L + 16L + Y 8n, bwd rows 16L (+ 8nd)
      r2c (L = n/2): as full with Y 4n (Y = |y~|^2 is even, Y_k = Y_{n-k}, and the kernel reads it only
                     at each mirror pair's primary element: the n/2 values Y_k, Y_{k+n/2})
      re (L = n/4, columns [0, N2/2) of the n/2-point transform, N1 = n/(2 N2) rows of N2 = 2^11):
                     rows 16L + the Nyquist column 16 N1; cols 16L + 16L + Y 4n (the pairs (Y_2k, Y_2k+1)
                     of its frequencies) + Nyquist 16 N1 read + 4 N1 written; bwd rows 16L + 4 N1"""
    variant = variant or fit_variant(n, parts_array)
    pb = 8 * n * d if parts_array else 0
    if variant in ("spectral", "spectral_fused"):
        # one shared set of 2^d spectra of K = n/2 + 1 doubles read once per launch, Y[:K] of every
        # problem, (4 + d) partials per problem and k block written (the fused kernel's level-1 group
        # sums, reads of the partials and the parameter / history updates are < 0.1% on top)
        K = n // 2 + 1
        nb, _, _ = spec_geometry(n, d, P)
        return {stage_names(variant)[0]: 8 * K * (2 ** d) + 8 * K * P + 8 * (4 + d) * nb * P}
    if variant == "re":
        L, N1 = n // 4, n // (2 * 2 ** re_row_log2())
        return {"k_fwd_rows": (16 * L + 16 * N1) * P, "k_fwd_cols": (32 * L + 4 * n + 20 * N1) * P,
                "k_bwd_rows": (16 * L + 4 * N1) * P}
    L = n // 2 if variant == "r2c" else n
    yb = 4 * n if variant == "r2c" else 8 * n
    return {"k_fwd_rows": (16 * L + pb) * P, "k_fwd_cols": (32 * L + yb) * P, "k_bwd_rows": (16 * L + pb) * P}


def wall_clock_khz(F, device):
    import ctypes
    khz = ctypes.c_int(0)
    F._native.call("fgp_wall_clock_khz", int(device.index or 0), ctypes.byref(khz))
    return khz.value


def roofline_fit_kernels(F, shifts, iters):
    """Per-kernel timing of the batched fit iteration as launched in the step (same engine, same grid),
    two ways:
      * device clock (fgp_nll_desc.stamps): first-workgroup start to last-wave end of every launch --
        the kernel duration rocprofv3 --kernel-trace reports; this is `avg_us` and prices `achieved`;
      * HIP events recorded on torch's current stream (the stream the kernels are launched on) around
        each launch behind a spin kernel that holds the stream while the host enqueues: kernel + the
        dependent-launch gap (`avg_us_events`)."""
    shifts.reset()
    gps = shifts.gps
    n = shifts.n
    dev = torch.device(gps[0].device)
    eng = F.batch.batched_engine(gps, iters)
    eng.run(0, 2)
    torch.cuda.synchronize()
    variant = "spectral" if eng.basis is not None else fit_variant(n, eng.gen is None)
    if variant == "spectral" and spec_fused(n, eng.d, eng.G):
        variant = "spectral_fused"
    names = stage_names(variant)
    ns = len(names)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(ns + 2)] for _ in range(iters)]
    fg = fit_grid(n, eng.G, variant, eng.d)      # (workgroups, threads) per fit launch
    # room for any grid the library picks (the host mirror of its geometry, fit_grid, is checked against the
    # workgroups that actually stamped below)
    grid = max(max(g for g, _ in fg.values()), 1 << 14)
    stamps = torch.zeros((iters, ns, grid, 5), dtype=torch.int64, device=dev)   # fgp_nll_desc.stamps
    torch.cuda._sleep(int(2.4e9 * 4e-4 * iters))
    fused = variant == "spectral_fused"
    for it in range(iters):
        e = ev[it]
        e[0].record()
        if fused:     # the step's own launch: one kernel per iteration (fgp_fit_run), stamped
            eng._nll.stamps = stamps[it, 0].data_ptr()
            eng.run(it, 1)
            e[1].record()
            e[2].record()
            continue
        for k in range(ns):
            eng._nll.stamps = stamps[it, k].data_ptr()
            eng.stage(k)
            e[k + 1].record()
        eng._nll.stamps = None
        eng.fit_step(it)
        e[ns + 1].record()
    eng._nll.stamps = None
    torch.cuda.synchronize()
    eng._nll.stamps = None
    khz = wall_clock_khz(F, dev)
    st = stamps.cpu()
    dur = []
    for k, name in enumerate(names):    # records [workgroup][start, wave ends...] of this launch's grid
        g, thr = fg[name]
        stamped = int((st[0, k, :, 0] > 0).sum())
        if stamped != g:                 # the library chose another geometry than the host mirror (small n)
            g = stamped
            fg[name] = (g, thr)
        sk = st[:, k, :g, :1 + thr // 64]
        assert g > 0 and bool((sk > 0).all()), "a fit launch did not write its device-clock stamps"
        dur.append((sk[..., 1:].amax((1, 2)) - sk[..., 0].amin(1)).double() * (1e3 / khz))
    dur_us = torch.stack(dur, 1)     # [iters, ns]
    us_ev = {name: 1e3 * sum(e[k].elapsed_time(e[k + 1]) for e in ev) / iters for k, name in enumerate(names)}
    if fused:
        # the per-launch events above include one counter reset per fgp_fit_run call; the step makes ONE
        # call for all its iterations -- time that (events around eng.run(0, iters)) for the iteration
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 2e-4))
        e0.record()
        eng.run(0, iters)
        e1.record()
        torch.cuda.synchronize()
        us_ev = {names[0]: 1e3 * e0.elapsed_time(e1) / iters}
        # the same call replayed from a hipGraph, as the timed step runs it (a replayed launch skips the eager
        # enqueue's per-packet work): HIP events around the replays, per iteration
        us_ev[names[0] + "@graph"] = graph_fit_us(eng, iters)
    us = {name: float(dur_us[:, k].mean()) for k, name in enumerate(names)}
    if not fused:
        us_ev["k_fit_reduce_step"] = 1e3 * sum(e[ns].elapsed_time(e[ns + 1]) for e in ev) / iters
        us["k_fit_reduce_step"] = us_ev["k_fit_reduce_step"]
    t_iter = sum(v for k, v in us_ev.items() if not k.endswith("@graph")) / 1e6
    return n, variant, us, us_ev, t_iter, khz


def graph_fit_us(eng, iters, reps=5):
    """Per-iteration time of eng.run(0, iters) (fgp_fit_run: one k_spec_tile per iteration + the final step)
    captured once into a hipGraph and replayed `reps` times between two HIP events; None when the capture fails."""
    try:
        cur = torch.cuda.current_stream()
        s = torch.cuda.Stream()
        s.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                eng.run(0, iters)
        cur.wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return 1e3 * e0.elapsed_time(e1) / (reps * iters)
    except Exception:                   # capture not possible here
        _clear_capture_error()
        return None


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # the repository
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06x_pmc_fit_kernels.json")
PMC_SQ_SUMMARY = os.path.join(ROOT, "profiles", "r06x_pmc_sq_fit_kernels.json")
ROCPROF_GRID_STATS = os.path.join(ROOT, "profiles", "r06x_bench_timed_region_stats.txt")
# the read floor of the spectral iteration's footprint: tools/stream_microbench.hip over the same 168 MB,
# re-read back to back, 24.0-24.3 us per pass (7.0 TB/s; profiles/r03v_stream_and_stamps.jsonl)
STREAM_FLOOR_US = 24.0
# FP64 VALU lane-operations per second: 256 CUs x 4 SIMDs x 16 FP64 lanes per clock x 2.4 GHz = 3.93e13
# (FP64 vector at half the FP32 vector rate of MI355X_MICROARCH.md, 157.3 TFLOP/s; 78.6 TFLOP/s FMA)
FP64_LANE_OPS_PEAK = 256 * 4 * 16 * 2.4e9
CPU_FIDELITY = os.path.join(ROOT, "profiles", "r02_cpu_fidelity.json")
# the prediction kernels (tools/predict_kernels.py: C4's batched post_mean / post_var, C5 per-output's post_mean):
# rocprofv3 kernel-trace summary and SQ counter pass
ROCPROF_PREDICT_STATS = os.path.join(ROOT, "profiles", "r06x_predict_kernel_grid_stats.txt")
PMC_SQ_PREDICT = os.path.join(ROOT, "profiles", "r06x_pmc_sq_predict.json")


def pmc_traffic(kernel, grid):
    """HBM bytes per launch of `kernel` at `grid` threads from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py over FETCH_SIZE / WRITE_SIZE passes of tools/fit_kernels.py, same kernels
    and grid; FETCH_SIZE x2 gfx950 correction), or None when absent."""
    try:
        summ = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None
    for k, v in summ.items():
        name, _, g = k.partition("|grid=")
        if name.split("<")[0].split("::")[-1] == kernel and g == str(grid) and "traffic_bytes" in v:
            return v["traffic_bytes"]
    return None


def _kernel_match(name, kernel):
    """`kernel` is a base name ("k_spec_tile": any template instance) or a full instance ("k_post_mean<0, 5, 1, 4>")."""
    full = name.split("::")[-1] if "<" not in name else name[name.index("k_"):] if "k_" in name else name
    if "<" in kernel:
        return full.replace(" ", "") == kernel.replace(" ", "")
    return name.split("<")[0].split("::")[-1] == kernel


def pmc_valu_insts(kernel, grid, path=None):
    """VALU wave-instructions per launch (SQ_INSTS_VALU) of `kernel` at `grid` threads from the committed
    SQ counter pass (tools/pmc_sq_summary.py over tools/fit_kernels.py; `path`: another summary, e.g. the
    prediction kernels' over tools/predict_kernels.py), or None when absent."""
    try:
        summ = json.load(open(path or PMC_SQ_SUMMARY))
    except (OSError, ValueError):
        return None
    for k, v in summ.items():
        name, _, g = k.partition("|grid=")
        if _kernel_match(name, kernel) and (grid is None or g == str(grid)) and "SQ_INSTS_VALU" in v:
            return v["SQ_INSTS_VALU"]
    return None


def rocprof_avg_us(kernel, grid, path=None):
    """Average duration of `kernel` at `grid` threads in the committed rocprofv3 --kernel-trace summary
    of this bench command (tools/kstats_grid.py over `rocprofv3 --kernel-trace --stats -- python3
    bench.py`; `path`: another summary), or None when absent."""
    try:
        lines = open(path or ROCPROF_GRID_STATS).read().splitlines()[1:]
    except OSError:
        return None
    for ln in lines:
        f = ln.split()
        if len(f) < 6:
            continue
        name = " ".join(f[:-5])
        if _kernel_match(name, kernel) and (grid is None or f[-5] == str(grid)):
            return float(f[-3])
    return None


def post_mean_ops_per_pair(d, nb):
    """FP64 VALU instructions per (test point, training point, output) of k_post_mean's folded-B4 loop
    (csrc/fgp_predict.hip; lattice, alpha = 2), read off its gfx950 ISA: per dimension v_add_f64 (x_t - z_i) and
    v_fma_f64 (u = t^2 - |t|) shared by the kernel's nb outputs, then per output v_fma_f64 (u^2 + c') and v_mul_f64
    into the product (less the first dimension's product by 1.0), and one v_fmac_f64 with the coefficient:
    (2 d + 2 d nb) / nb -- 4 d for one output."""
    return (2.0 * d + 2.0 * d * nb) / nb


def roofline_post_mean(kernel, grid, pairs, d, nb, stats=None, sq=None, live_ms=None, launches=1):
    """FP64-VALU roofline of a posterior-mean launch (abstract_gp.py:352-380; matrix-free cross-kernel
    contraction): `pairs` (test point, training point, output) triples per launch x post_mean_ops_per_pair
    lane-operations over the rocprofv3 average duration, against the FP64 VALU issue peak; beside it the
    measured SQ_INSTS_VALU x 64 lanes over the same duration (every VALU instruction, address and loop
    arithmetic included)."""
    us = rocprof_avg_us(kernel, grid, stats)
    ops = post_mean_ops_per_pair(d, nb)
    out = {"bound": "fp64 valu", "kernel": kernel, "pairs_per_launch": pairs, "ops_per_pair": ops,
           "op_model": "per dimension v_add_f64 + v_fma_f64 shared by %d output(s), v_fma_f64 + v_mul_f64 per output, "
                       "one v_fmac_f64 per output (gfx950 ISA of the folded-B4 loop)" % nb,
           "peak": FP64_LANE_OPS_PEAK, "unit": "FP64 lane-ops/s", "launches_per_step": launches,
           "avg_us_source": "rocprofv3 --kernel-trace average, %s" % os.path.relpath(stats or ROCPROF_GRID_STATS, ROOT)}
    if us is None:
        return out
    ach = pairs * ops / (us * 1e-6)
    out.update({"avg_us": us, "achieved": ach, "frac": ach / FP64_LANE_OPS_PEAK})
    vi = pmc_valu_insts(kernel, grid, sq)
    if vi is not None:
        out["valu"] = {"insts_per_launch": vi, "frac": vi * 64 / (us * 1e-6) / FP64_LANE_OPS_PEAK,
                       "source": os.path.relpath(sq or PMC_SQ_SUMMARY, ROOT) + " (SQ_INSTS_VALU)"}
    if live_ms is not None:
        out["phase_ms_live"] = live_ms
    return out


SECONDARY_STATS = os.path.join(ROOT, "profiles", "r06k_secondary_stats.json")
FP64_MFMA_PEAK_FLOPS = 78.6e12       # MI355X FP64 matrix peak (spec; = the FP64 vector FMA rate)


def secondary_rooflines(case, n, d, outputs, n_mean, fit_iters):
    """Rooflines of a secondary line's kernels, priced on the committed rocprofv3 trace + PMC passes
    of the same steps (tools/secondary_profile.sh -> tools/secondary_kernels.py, profiles/r06k_secondary_stats.json;
    durations: the kernel trace's per-launch averages; traffic: FETCH_SIZE x2 (gfx950) + WRITE_SIZE per launch).
    Returns [primary, others...] (primary = the line's longest kernel per step) or []."""
    try:
        st = json.load(open(SECONDARY_STATS))
    except (OSError, ValueError):
        return []
    tr = st["trace"].get(case)
    if not tr:
        return []
    src = os.path.relpath(SECONDARY_STATS, ROOT)

    def find(prefix):
        for k, v in tr.items():
            if k.startswith(prefix):
                return k, v
        return None, None

    def counters(k):
        f = st.get("fetch_kb", {}).get(case, {}).get(k)
        w = st.get("write_kb", {}).get(case, {}).get(k)
        q = st.get("sq_insts_valu", {}).get(case, {}).get(k)
        return (None if f is None or w is None else 2.0 * f * 1024 + w * 1024), q

    def hbm(k, v, alg, what):
        traffic, q = counters(k)
        ach = alg / (v["avg_us"] * 1e-6) / 1e9
        r = {"bound": "hbm", "kernel": k.split("|")[0], "grid_threads": int(k.split("=")[-1]), "algorithmic_bytes": alg,
             "bytes_model": what, "avg_us": v["avg_us"], "launches_per_step": v["launches_per_step"],
             "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
             "source": src}
        if q is not None:
            r["valu_frac"] = q * 64 / (v["avg_us"] * 1e-6) / FP64_LANE_OPS_PEAK
        return r

    K = n // 2 + 1 if case != "C3" else n
    out = []
    if case in ("C2", "C3"):
        k, v = find("k_spec_persist")
        if k is not None:
            traffic, q = counters(k)
            ach = q * 64 / (v["avg_us"] * 1e-6) if q is not None else None
            lds = 8 * K * (2 ** d + 1)        # the spectra + Y, LDS-resident, read once per iteration
            out.append({"bound": "latency (one grid barrier + reduction + Rprop step per iteration)", "kernel": k.split("|")[0],
                        "grid_threads": int(k.split("=")[-1]), "avg_us": v["avg_us"], "iterations": fit_iters + 1,
                        "iteration_us": v["avg_us"] / (fit_iters + 1), "achieved": ach, "peak": FP64_LANE_OPS_PEAK,
                        "unit": "FP64 lane-ops/s (SQ_INSTS_VALU x 64)", "frac": None if ach is None else ach / FP64_LANE_OPS_PEAK,
                        "lds_bytes_per_iteration": lds, "hbm_traffic_per_launch": traffic,
                        "note": "the whole 51-iteration fit in one launch (fgp_fit_persist): spectra + Y stay in LDS, so "
                                "neither HBM nor VALU bounds the iteration; its time is the in-kernel barrier chain",
                        "source": src})
    if case in ("C5", "C5 mixed"):
        k, v = find("Cijk_")
        if k is not None:
            flops = 2.0 * n_mean * n * outputs / v["launches_per_step"]
            ach = flops / (v["avg_us"] * 1e-6)
            out.append({"bound": "mfma (fp64)", "kernel": "library DGEMM (post_mean: kernel rows x coefficients)",
                        "kernel_symbol": k.split("|")[0][:80], "flops_per_launch": flops,
                        "flops_model": "2 N n B over its launches per step", "avg_us": v["avg_us"],
                        "launches_per_step": v["launches_per_step"], "achieved": ach / 1e12, "peak": FP64_MFMA_PEAK_FLOPS / 1e12,
                        "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_FLOPS, "traffic": counters(k)[0], "source": src})
        k, v = find("k_inv_cols_c2r")
        if k is not None:
            out.append(hbm(k, v, 32.0 * (n // 2) * outputs, "coefficients, column pass: 16 (n/2) B read + 16 (n/2) B written"))
        k, v = find("k_inv_rows_c2r")
        if k is not None:
            out.append(hbm(k, v, (16.0 * (n // 2) + 8.0 * n) * outputs, "coefficients, row pass: 16 (n/2) B read + 8 n B written"))
        k, v = find("k_spec_persist")
        if k is not None:
            traffic, q = counters(k)
            out.append({"bound": "latency (single-launch fit)", "kernel": k.split("|")[0], "avg_us": v["avg_us"],
                        "iteration_us": v["avg_us"] / (fit_iters + 1), "frac": None if q is None else
                        q * 64 / (v["avg_us"] * 1e-6) / FP64_LANE_OPS_PEAK, "unit": "FP64 VALU fraction", "source": src})
    if case == "C5 per-output":
        k, v = find("k_spec_tile")
        if k is not None:
            out.append(hbm(k, v, 8.0 * K * (2 ** d) + 8.0 * K * outputs,
                           "one fit iteration of %d problems sharing the spectra: 2^d spectra + Y of every problem, "
                           "8 K bytes each (K = n/2 + 1)" % outputs))
        k, v = find("k_spec_post_var")
        if k is not None:
            traffic, q = counters(k)
            if q is not None:
                ach = q * 64 / (v["avg_us"] * 1e-6)
                out.append({"bound": "fp64 valu", "kernel": k.split("|")[0], "avg_us": v["avg_us"],
                            "launches_per_step": v["launches_per_step"], "achieved": ach, "peak": FP64_LANE_OPS_PEAK,
                            "unit": "FP64 lane-ops/s (SQ_INSTS_VALU x 64)", "frac": ach / FP64_LANE_OPS_PEAK,
                            "traffic": traffic, "note": "post_var of the %d problems by linearity of the test points' row "
                            "spectra: per (problem, test point, frequency) the 2^d-term polynomial" % outputs,
                            "source": src})
    out.sort(key=lambda r: -(r.get("avg_us", 0) * r.get("launches_per_step", 1)))
    return out
