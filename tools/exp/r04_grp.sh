#!/bin/bash
# A/B of the level-1 group size (kSpecGroup 32 default, 16, 64 experiment builds): fused C4 iteration stamps
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04grp}
mkdir -p $OUT
set -e
for rep in 1 2; do
  for v in def g16 g64; do
    if [ $v = def ]; then unset FGP_LIB_PATH; else export FGP_LIB_PATH=$PWD/fastgaussianprocesses_amd/_lib/exp/libfgp_$v.so; fi
    echo "{\"variant_lib\": \"$v\", \"rep\": $rep}" >> $OUT/stamps.jsonl
    timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 >> $OUT/stamps.jsonl 2>> $OUT/stamps.err
  done
done
unset FGP_LIB_PATH
export FGP_LIB_PATH=$PWD/fastgaussianprocesses_amd/_lib/exp/libfgp_g16.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_spectral.py -m gpu -q -x --timeout 150 --timeout-method thread > $OUT/pytest_g16.log 2>&1
tail -2 $OUT/pytest_g16.log
grep -h -E "variant_lib|fused" $OUT/stamps.jsonl | cut -c1-200
