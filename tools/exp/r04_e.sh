#!/bin/bash
# parity subset, C4 iteration stamps, single-launch fit stamps, then the full bench with --graph
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04e}
mkdir -p $OUT
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_gp.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -6 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
set -e
timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 > $OUT/stamps.jsonl 2> $OUT/stamps.err; cat $OUT/stamps.jsonl
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl
timeout -k 10 600 python -u bench.py --graph $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
python - <<PY
import json
d = json.load(open("$OUT/bench.json"))
print(d["value"], d["ms_per_step"], d["phases_ms"], d.get("graph"))
for s in d.get("secondary") or []:
    print(s["config"]["workload"][:40], round(s["ms_per_step"], 3), s.get("graph"))
print([(c["benchmark"], c["class"][:14], round(c["s_per_step"] * 1e6, 1)) for c in (d.get("paper") or {}).get("configs", [])])
PY
if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
