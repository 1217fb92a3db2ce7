#!/bin/bash
# Stamps of the in-tree build vs an experiment build (EXPLIB).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03s6}
mkdir -p $OUT
for L in "" $EXPLIB; do
  echo "{\"lib\": \"${L:-in-tree}\"}" >> $OUT/stamps.jsonl
  FGP_LIB_PATH=$L timeout -k 10 200 python -u tools/exp_spec_stamps.py --iters 20 >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
done
cat $OUT/stamps.jsonl
echo done
