#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04ab3}
mkdir -p $OUT
set -e
L=fastgaussianprocesses_amd/_lib
for rep in 1 2; do
  for v in hip pm4 pm1; do
    if [ $v = hip ]; then lib=$L/libfgp_hip.so; else lib=$L/exp/libfgp_$v.so; fi
    FGP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-secondary --no-multitask --no-paper --no-cpu-baseline > $OUT/b_$v$rep.json 2> $OUT/b_$v$rep.err
    python -c "import json;d=json.load(open('$OUT/b_$v$rep.json'));print('$v', $rep, round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['phases_ms'].items()})"
  done
done
echo done
