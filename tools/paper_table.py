"""DESIGN.md's paper table from a bench line's `paper` section:

    python tools/paper_table.py profiles/r04u_bench.json
"""
import json
import sys

b = json.load(open(sys.argv[1]))
rows = {}
for c in b["paper"]["configs"]:
    col = (c["gp"].startswith("SI"), c["data"] != "f")
    rows.setdefault("%s d=%d" % (c["benchmark"], c["d"]), {})[col] = c
order = [(True, False), (True, True), (False, False), (False, True)]
for name, cols in rows.items():
    cells = []
    for k in order:
        c = cols.get(k)
        cells.append("%.1e (paper %.1e)" % (c["s_per_step"], c["paper_s_per_step"]) if c else "--")
    print("| %s | %s |" % (name, " | ".join(cells)))
