"""Per-(kernel, grid) durations of the launches inside bench.py's TIMED region, from a rocprofv3 kernel trace of
the bench command itself (`rocprofv3 --kernel-trace -- python3 bench.py ...`): bench.py brackets its timed loop
with two k_clock_stamp launches (outside the timed interval), so the kernels between the first two k_clock_stamp
launches of the trace are the timed steps -- with a graph, the replays.  Same table format as kstats_grid.py (what
bench.rocprof_avg_us reads), plus a header line naming the region.

    python tools/timed_region_stats.py <kernel_trace.csv> [top]
"""
import collections
import csv
import sys


def timed_rows(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_clock_stamp" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit("no timed-region markers (two k_clock_stamp launches) in %s" % path)
    return rows[marks[0] + 1:marks[1]], rows[marks[0]], rows[marks[1]]


def main():
    rows, m0, m1 = timed_rows(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[(name, r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values())
    span = int(m1["Start_Timestamp"]) - int(m0["End_Timestamp"])
    print("%-90s %9s %6s %10s %10s %7s" % ("kernel", "grid", "calls", "avg_us", "med_us", "pct"))
    for (name, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        s = sorted(v)
        print("%-90s %9s %6d %10.1f %10.1f %6.2f%%" % (name[:90], g, len(v), sum(v) / len(v) / 1e3, s[len(s) // 2] / 1e3,
                                                     100.0 * sum(v) / tot))
    print("timed region: %d launches, kernel time %.3f ms, marker to marker %.3f ms" % (len(rows), tot / 1e6, span / 1e6))


if __name__ == "__main__":
    main()
