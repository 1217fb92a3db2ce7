#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) over the fit kernels (tools/fit_kernels.py), one run each.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcf}
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 tools/fit_kernels.py > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 tools/fit_kernels.py > $OUT/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
echo pmc done
