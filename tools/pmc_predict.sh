#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) over the prediction kernels (tools/predict_kernels.py), one run each.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcp}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcp_fetch -o fetch -- python3 tools/predict_kernels.py > $OUT/pmcp_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcp_write -o write -- python3 tools/predict_kernels.py > $OUT/pmcp_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmcp_sq -o sq -- python3 tools/predict_kernels.py > $OUT/pmcp_sq.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 tools/predict_kernels.py > $OUT/trace.log 2>&1
echo pmc done
