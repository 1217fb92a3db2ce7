#!/bin/bash
# A/B of the spectral blocks' minimum chunk count on the C2 / C3 single-launch fits (needs the FGP_SPEC_MINC knob of the r05z A/B build, since reverted: profiles/r05z_persist_minc_ab.json): kernel trace
# of tools/prof_single.py per setting
export TMPDIR=/tmp
OUT=gpurun_out/minc
mkdir -p $OUT
set -e
for m in 4 2 1 8; do
  for fam in lattice net; do
    FGP_SPEC_MINC=$m timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/m${m}_$fam -o t -- python3 tools/prof_single.py --family $fam --reps 4 > $OUT/m${m}_$fam.log 2>&1
  done
done
echo done
