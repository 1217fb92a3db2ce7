#!/bin/bash
# Round-3 session-2 call: spectral-iteration stamps for the in-tree build and the ring-depth experiment
# builds, then the full round check (tools/r03_round.sh).  Every GPU step has its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03u}
mkdir -p $OUT
for L in "" fastgaussianprocesses_amd/_lib/exp/libfgp_ring3.so fastgaussianprocesses_amd/_lib/exp/libfgp_ring4.so; do
  echo "lib=${L:-in-tree}" >> $OUT/stamps.jsonl
  FGP_LIB_PATH=$L timeout -k 10 200 python -u tools/exp_spec_stamps.py >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
done
cat $OUT/stamps.jsonl
if [ -z "$NOROUND" ]; then TAG=${TAG:-r03u} bash tools/r03_round.sh; fi
