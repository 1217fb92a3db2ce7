"""Summarise a rocprofv3 --pmc pass of SQ_* counters per kernel and grid (per-launch averages),
plus the VGPR / AGPR / scratch / LDS resources of each kernel.

  python tools/pmc_sq_summary.py sq_counter_collection.csv > out.json
"""
import collections
import csv
import json
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    res = {}
    for row in csv.DictReader(open(sys.argv[1])):
        key = "%s|grid=%s" % (row["Kernel_Name"].split("(")[0].replace("void ", ""), row.get("Grid_Size", ""))
        vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
        res[key] = {"vgpr": int(row["VGPR_Count"]), "agpr": int(row["Accum_VGPR_Count"]),
                    "scratch": int(row["Scratch_Size"]), "lds": int(row["LDS_Block_Size"])}
    out = {}
    for k in sorted(vals, key=lambda k: -sum(vals[k].get("SQ_BUSY_CYCLES", [0]))):
        out[k] = {c: sum(v) / len(v) for c, v in sorted(vals[k].items())}
        w = out[k].get("SQ_WAVES")
        if w:
            out[k]["valu_per_wave"] = out[k].get("SQ_INSTS_VALU", 0.0) / w
            out[k]["lds_per_wave"] = out[k].get("SQ_INSTS_LDS", 0.0) / w
        out[k]["resources"] = res[k]
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
