"""Per-case kernel statistics of tools/secondary_kernels.py's rocprofv3 trace (kernel_trace.csv): the launches between
each pair of k_clock_stamp markers, per (kernel, grid): launches per step, average duration (us), total per step.
With --pmc FETCH.csv WRITE.csv SQ.csv (counter_collection files of separate --pmc passes of the same tool): HBM bytes
per launch (FETCH_SIZE x2 on gfx950 + WRITE_SIZE) and SQ_INSTS_VALU per launch.

    python tools/secondary_stats.py TRACE.csv [--steps 3] [--pmc FETCH.csv WRITE.csv SQ.csv] > stats.json
"""
import collections
import csv
import json
import sys

CASES = ("C2", "C3", "C5", "C5 per-output", "C5 mixed")


def short(name):
    n = name.split("(")[0].replace("void ", "").strip()
    return n.split("fgp::")[-1] if "fgp::" in n else n[:80]


def segments(rows, key_name):
    """Rows in start order split at the marker launches (k_clock_stamp): [case] -> rows."""
    out, cur, inside = [], None, False
    for r in rows:
        if "k_clock_stamp" in r[key_name]:
            if not inside:
                cur, inside = [], True
            else:
                out.append(cur)
                inside = False
            continue
        if inside:
            cur.append(r)
    return out


def trace_stats(path, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    res = {}
    for case, seg in zip(CASES, segments(rows, "Kernel_Name")):
        agg = collections.defaultdict(list)
        for r in seg:
            grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) * int(r.get("Grid_Size_Y", 1) or 1) * \
                int(r.get("Grid_Size_Z", 1) or 1)
            agg["%s|grid=%d" % (short(r["Kernel_Name"]), grid)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        k = {name: {"launches_per_step": len(v) / steps, "avg_us": sum(v) / len(v), "us_per_step": sum(v) / steps}
             for name, v in agg.items()}
        res[case] = dict(sorted(k.items(), key=lambda kv: -kv[1]["us_per_step"]))
    return res


def pmc_stats(path, counter, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r.get("Start_Timestamp", r.get("Dispatch_Id", 0)) or 0))
    res = {}
    # the pmc csv has one row per (dispatch, counter); the markers are dispatches too
    seq = []
    for r in rows:
        seq.append(r)
    for case, seg in zip(CASES, segments(seq, "Kernel_Name")):
        agg = collections.defaultdict(list)
        for r in seg:
            if r.get("Counter_Name") != counter:
                continue
            grid = r.get("Grid_Size", "")
            agg["%s|grid=%s" % (short(r["Kernel_Name"]), grid)].append(float(r["Counter_Value"]))
        res[case] = {k: sum(v) / len(v) for k, v in agg.items()}
    return res


def main():
    a = sys.argv[1:]
    steps = int(a[a.index("--steps") + 1]) if "--steps" in a else 3
    out = {"trace": trace_stats(a[0], steps)}
    if "--pmc" in a:
        i = a.index("--pmc")
        f, w, q = a[i + 1:i + 4]
        out["fetch_kb"] = pmc_stats(f, "FETCH_SIZE", steps)
        out["write_kb"] = pmc_stats(w, "WRITE_SIZE", steps)
        out["sq_insts_valu"] = pmc_stats(q, "SQ_INSTS_VALU", steps)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
