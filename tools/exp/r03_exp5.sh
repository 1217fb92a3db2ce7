#!/bin/bash
# Spectral-path parity tests + stamps + bench (no CPU baseline), each step time-limited.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03x}
mkdir -p $OUT
rc=0
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_gp.py tests/test_gpu_configs.py tests/test_gpu_multioutput.py} -m gpu -q ${PYX--x} --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -8 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u tools/exp_spec_stamps.py > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.jsonl
timeout -k 10 600 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<PY
import json
d=json.load(open("$OUT/bench.json"))
print(d["value"], d["ms_per_step"], d["phases_ms"])
print({k: (round(v["avg_us"],1), round(v["avg_us_events"],1)) for k, v in d["roofline"]["kernels"].items()})
for s in d["secondary"] or []: print(s["config"]["workload"][:50], round(s["ms_per_step"],3), s["phases_ms"])
for c in (d.get("paper") or {}).get("configs", []): print(c["benchmark"], c["gp"][:10], c["data"], c["tasks"], c["iterations"], "%.2e" % c["s_per_step"], c["paper_s_per_step"], c["class"])
PY
echo done
