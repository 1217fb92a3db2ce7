"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (per-launch averages).

  python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv > out.json

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B streaming stores.  Both are in KB.
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row.get("Counter_Name") != counter:
            continue
        name = row["Kernel_Name"]
        key = "%s|grid=%s" % (name.split("(")[0].replace("void ", ""), row.get("Grid_Size", ""))
        vals[key].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k)
        wb = write.get(k)
        out[k] = {"fetch_bytes_corrected": None if fb is None else 2.0 * fb * 1024,
                  "write_bytes": None if wb is None else wb * 1024,
                  "dispatches": max(nf.get(k, 0), nw.get(k, 0))}
        if fb is not None and wb is not None:
            out[k]["traffic_bytes"] = out[k]["fetch_bytes_corrected"] + out[k]["write_bytes"]
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
