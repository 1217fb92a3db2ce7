#!/bin/bash
# Row-length sweep of the real-even fit kernels (FGP_RE_P2 = 10, 11, 12): the bench-path parity test
# at each split, then the bench line (no CPU baseline / secondary configs).
set -e
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
for p in ${P2S:-10 11 12}; do
  FGP_RE_P2=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_configs.py -k "bench_step or half_length_fit" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_p$p.log 2>&1
  tail -1 $OUT/pytest_p$p.log
  FGP_RE_P2=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $OUT/bench_p$p.json 2> $OUT/bench_p$p.err
  python -c "import json,sys; d=json.load(open('$OUT/bench_p$p.json')); print($p, d['value'], d['phases_ms']['fit'], {k: round(v['avg_us'],1) for k, v in d['roofline']['kernels'].items()})"
done
