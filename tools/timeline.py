"""Split a rocprofv3 kernel trace into fit segments (batched fit kernels) and other segments:
span, GPU-busy time and kernel count of each.   python tools/timeline.py <kernel_trace.csv> [grid]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
fit_grid = sys.argv[2] if len(sys.argv) > 2 else "524288"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
segs = []
cur = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    g = r["Grid_Size_X"]
    fit = ("fgp::k_" in name and g == fit_grid) or "k_fit_reduce_step" in name
    tag = "fit" if fit else "other"
    if cur is None or cur["tag"] != tag:
        cur = {"tag": tag, "s": s, "e": e, "busy": 0, "k": 0, "names": {}}
        segs.append(cur)
    cur["e"] = e
    cur["busy"] += e - s
    cur["k"] += 1
    short = name.split("<")[0][-40:]
    cur["names"][short] = cur["names"].get(short, 0) + (e - s)
for sg in segs:
    top = sorted(sg["names"].items(), key=lambda x: -x[1])[:4]
    print("%-5s t=%9.2f ms span %8.3f ms busy %8.3f ms kernels %4d  %s" % (
        sg["tag"], (sg["s"] - t0) / 1e6, (sg["e"] - sg["s"]) / 1e6, sg["busy"] / 1e6, sg["k"],
        ", ".join("%s %.0fus" % (n, v / 1e3) for n, v in top) if sg["tag"] == "other" else ""))
