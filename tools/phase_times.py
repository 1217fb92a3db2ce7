"""Phase breakdown of the real-even row kernels from an experiment build with -DFGP_EXP_PHASES
(tools/build_exp.sh FGP_EXP_PHASES phases): thread 0 of every workgroup stamps the wall clock at the
kernel's phase marks; prints the mean (and 90th percentile) time from the kernel's first stamp.

    FGP_LIB_PATH=.../libfgp_phases.so python tools/phase_times.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.set_default_dtype(torch.float64)


def main():
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    sh = bench.Shifts(F, 5, 2 ** 20, [1000 + s for s in range(8)], dev)
    sh.reset()
    eng = F.batch.batched_engine(sh.gps, 4)
    eng.run(0, 2)
    grid = 8 * (2 ** 20 // 4096) + 8
    khz = bench.wall_clock_khz(F, dev)
    out = {}
    for stage, name in ((0, "k_fwd_rows_re"), (2, "k_bwd_rows_re")):
        buf = torch.zeros((grid, 16), dtype=torch.int64, device=dev)
        for rep in range(3):
            eng.stage(0)
            eng.stage(1)
            eng._nll.stamps = buf.data_ptr() if True else None
            if stage == 0:
                eng._nll.stamps = buf.data_ptr()
                eng.stage(0)
                eng._nll.stamps = None
                eng.stage(1)
                eng.stage(2)
            else:
                eng._nll.stamps = None
                eng.stage(0)
                eng.stage(1)
                eng._nll.stamps = buf.data_ptr()
                eng.stage(2)
                eng._nll.stamps = None
            eng.fit_step(0)
        torch.cuda.synchronize()
        st = buf.cpu().double()
        used = st[:, 0] > 0
        st = st[used]
        t0 = st[:, 0].min()
        ph = {}
        for k in range(1, 16):
            col = st[:, k]
            if not bool((col > 0).any()):
                continue
            rel = (col - st[:, 0]) * (1e3 / khz)
            ph["P%d" % k] = {"mean_us": round(float(rel.mean()), 2), "p90_us": round(float(rel.quantile(0.9)), 2)}
        start = (st[:, 0] - t0) * (1e3 / khz)
        ph["start_spread_us"] = {"mean": round(float(start.mean()), 2), "max": round(float(start.max()), 2)}
        last = max(k for k in range(1, 16) if bool((st[:, k] > 0).any()))
        end = (st[:, last] - t0) * (1e3 / khz)
        idx = torch.nonzero(used).reshape(-1)
        ph["end_us"] = {"mean": round(float(end.mean()), 2), "p50": round(float(end.quantile(0.5)), 2),
                        "p90": round(float(end.quantile(0.9)), 2), "max": round(float(end.max()), 2)}
        ph["end_by_xcd"] = [round(float(end[(idx % 8) == x].mean()), 2) for x in range(8)]
        pairs = int(idx.max()) // 8 + 1
        ph["end_jp0"] = round(float(end[(idx % pairs) == 0].mean()), 2)
        ph["end_by_block_octile"] = [round(float(end[(idx * 8 // (int(idx.max()) + 1)) == o].mean()), 2) for o in range(8)]
        ph["dur_by_block_octile"] = [round(float((end - start)[(idx * 8 // (int(idx.max()) + 1)) == o].mean()), 2) for o in range(8)]
        ph["start_by_block_octile"] = [round(float(start[(idx * 8 // (int(idx.max()) + 1)) == o].mean()), 2) for o in range(8)]
        out[name] = ph
    print(json.dumps(out))


if __name__ == "__main__":
    main()
