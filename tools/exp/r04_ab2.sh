#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04ab2}
mkdir -p $OUT
set -e
L=fastgaussianprocesses_amd/_lib
for rep in 1 2; do
  for v in def gen pf0; do
    case $v in
      def) E="";; gen) E="FGP_SPEC_BASIS_GEN=1";; pf0) E="FGP_LIB_PATH=$L/exp/libfgp_pf0.so";;
    esac
    env $E timeout -k 10 300 python -u bench.py --no-secondary --no-multitask --no-paper --no-cpu-baseline > $OUT/b_$v$rep.json 2> $OUT/b_$v$rep.err
    python -c "import json;d=json.load(open('$OUT/b_$v$rep.json'));print('$v', $rep, round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['phases_ms'].items()}, round(d['roofline']['avg_us_device_clock'],2), round(d['roofline']['avg_us_events'],2))"
  done
done
echo done
