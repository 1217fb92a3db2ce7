#!/bin/bash
# A/B of experiment builds: bench.py (no CPU baseline) with each FGP_LIB_PATH in $LIBS (space-separated
# names under fastgaussianprocesses_amd/_lib/exp/, "default" = the in-tree library), one line each.
set -e
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for L in ${LIBS:-default}; do
  # "default" = the in-tree library, "nomix" = the same with FGP_FIT_MIXED=0
  MIX=1
  if [ "$L" = default ]; then P=""; elif [ "$L" = nomix ]; then P=""; MIX=0; else P=fastgaussianprocesses_amd/_lib/exp/libfgp_$L.so; fi
  FGP_FIT_MIXED=$MIX FGP_LIB_PATH=$P timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_$L.json 2> $OUT/bench_$L.err
  python -c "import json; d=json.load(open('$OUT/bench_$L.json')); print('$L', d['value'], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms'].items()}); print({k: (round(v['avg_us'],1), round(v['avg_us_events'],1)) for k, v in d['roofline']['kernels'].items()})"
done
