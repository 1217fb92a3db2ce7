#!/bin/bash
# PMC passes (one counter group per run) over a kernel driver script: SQ and FETCH/WRITE.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
DRV=${DRV:-tools/fit_kernels.py}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 $DRV > $OUT/pmc_sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 $DRV > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 $DRV > $OUT/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $DRV > $OUT/kt.log 2>&1
python3 tools/pmc_sq_summary.py $(find $OUT/pmc_sq -name "*counter_collection.csv" | head -1) > $OUT/sq.json
python3 tools/pmc_summary.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) > $OUT/fw.json 2>/dev/null || true
python3 - <<PY
import json
sq=json.load(open("$OUT/sq.json"))
for k,v in sq.items():
    if "spec" in k or "fit" in k:
        print(k[:70], {c: round(v[c]) if isinstance(v[c], float) and v[c] > 100 else v[c] for c in v if c != "resources"})
PY
echo done
