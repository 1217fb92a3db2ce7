#!/bin/bash
# Spectral tile kernel decomposition: stamps of the in-tree build and of the experiment builds
# sx1 (streaming only), sx2 (compute only, no loads), sx3 (compute without the spectra's LDS reads).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03w}
mkdir -p $OUT
for L in "" fastgaussianprocesses_amd/_lib/exp/libfgp_sx1.so fastgaussianprocesses_amd/_lib/exp/libfgp_sx2.so fastgaussianprocesses_amd/_lib/exp/libfgp_sx3.so; do
  echo "{\"lib\": \"${L:-in-tree}\"}" >> $OUT/stamps.jsonl
  FGP_LIB_PATH=$L timeout -k 10 200 python -u tools/exp_spec_stamps.py --iters 10 >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
done
cat $OUT/stamps.jsonl
echo done
