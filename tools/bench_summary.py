"""One-screen summary of a bench.py JSON line (the headline, its timing sources, the secondary lines' eager / graph
rates and phases): python tools/bench_summary.py <bench output file>"""
import json
import sys


def main(path):
    d = json.loads([ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1])
    print("C4 %.4g points/s  %.3f ms/step (graph)  eager %.3f ms" % (d["value"], d["ms_per_step"],
                                                                      d["timing"]["ms_per_step_eager"]))
    r = d["roofline"]
    print("roofline %s frac %.3f avg_us %.1f (device clock %.1f, events %.1f, graph events %s)" % (
        r["kernel"], r["frac"], r["avg_us"], r["avg_us_device_clock"], r["avg_us_events"], r.get("avg_us_graph_events")))
    print("phases", {k: round(v, 3) for k, v in d["phases_ms"].items()})
    for s in d.get("secondary") or []:
        g = s.get("graph") or {}
        print("%-40s %.4g  %.3f ms (eager %s)  err=%s" % (s["config"]["workload"][:40], s["value"] or 0, s["ms_per_step"],
                                                         g.get("eager_ms_per_step"), s.get("error")))
        print("    eager phases", {k: round(v, 3) for k, v in (s.get("phases_ms") or {}).items()})
        print("    graph phases", g.get("phases_ms"))
        if s.get("roofline"):
            print("    roofline", s["roofline"])


if __name__ == "__main__":
    main(sys.argv[1])
