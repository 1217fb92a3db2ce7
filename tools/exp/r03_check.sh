#!/bin/bash
# Round-3 GPU check: the spectral-path parity tests, the whole GPU suite, smoke, a bench line.
# Every GPU step has its own time limit; the script stops at a crash or timeout.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
rc=0
timeout -k 10 300 python -u -m pytest ${SPEC_TESTS:-tests/test_gpu_spectral.py} -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_spectral.log 2>&1 || rc=$?
tail -15 $OUT/pytest_spectral.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
if [ -z "$NOSUITE" ]; then
  rc=0
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
  tail -25 $OUT/pytest_gpu.log
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || tail -5 $OUT/smoke.log
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['phases_ms']); print({k: (round(v['avg_us'],1), round(v['avg_us_events'],1)) for k, v in d['roofline']['kernels'].items()}); print([(s['config']['workload'][:40], round(s['ms_per_step'],3), s['phases_ms']) for s in (d['secondary'] or [])])"
echo done
