#!/bin/bash
# A/B of experiment builds (tools/build_exp.sh) on the C4 fit iteration: exp_spec_stamps.py per library,
# interleaved, each with its own time limit.  VARIANTS="name ..." (default: the in-tree build and every exp lib).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04ab}
mkdir -p $OUT
L=fastgaussianprocesses_amd/_lib
for rep in 1 2; do
  for v in ${VARIANTS:-hip $(ls $L/exp/ | sed -n 's/^libfgp_\(.*\)\.so$/\1/p')}; do
    if [ "$v" = hip ]; then lib=$L/libfgp_hip.so; else lib=$L/exp/libfgp_$v.so; fi
    echo "{\"build\": \"$v\", \"rep\": $rep}" >> $OUT/ab.jsonl
    FGP_LIB_PATH=$lib timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 >> $OUT/ab.jsonl 2>> $OUT/ab.err
  done
done
cat $OUT/ab.jsonl
