"""Per-(kernel, grid) duration statistics from a rocprofv3 kernel trace (the stats CSV averages a
kernel over every grid it ran at).   python tools/kstats_grid.py <kernel_trace.csv> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[(name, r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in agg.values())
print("%-90s %9s %6s %10s %10s %7s" % ("kernel", "grid", "calls", "avg_us", "med_us", "pct"))
for (name, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    s = sorted(v)
    print("%-90s %9s %6d %10.1f %10.1f %6.2f%%" % (name[:90], g, len(v), sum(v) / len(v) / 1e3, s[len(s) // 2] / 1e3,
                                                 100.0 * sum(v) / tot))
print("total GPU time %.1f ms" % (tot / 1e6))
