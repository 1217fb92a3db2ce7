#!/bin/bash
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
for S in 8 1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $OUT/sq$S -o sq -- python3 tools/fit_kernels.py --shifts $S > $OUT/sq$S.log 2>&1
python3 tools/pmc_sq_summary.py $(find $OUT/sq$S -name "*counter_collection.csv" | head -1) > $OUT/sq$S.json
python3 - <<PY
import json
sq=json.load(open("$OUT/sq$S.json"))
for k,v in sq.items():
    if "spec_tile" in k:
        print("$S", k[:60], {c: round(v[c]) if isinstance(v[c], float) and v[c] > 100 else v[c] for c in v if c != "resources"})
PY
done
