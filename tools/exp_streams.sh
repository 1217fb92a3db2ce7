#!/bin/bash
# GPU suite once, then the fit iteration time with 1, 2 and 4 problem groups on their own streams.
set -e
OUT=gpurun_out/${TAG:-streams}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for S in 1 2 4; do
  FGP_FIT_STREAMS=$S timeout -k 10 200 python -u tools/stage_times.py --tag s$S >> $OUT/times.jsonl 2> $OUT/err_s$S.log
done
cat $OUT/times.jsonl
for S in 1 2; do
  FGP_FIT_STREAMS=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $OUT/bench_s$S.json 2> $OUT/bench_s$S.err
  python -c "import json; d=json.load(open('$OUT/bench_s$S.json')); print('S=$S', d['value'], d['phases_ms'])"
done
