#!/bin/bash
# Multitask GPU tests (no -x) + the generic-loop NaN diagnostic.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03mt}
mkdir -p $OUT
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_multitask.py -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
grep -E "^E  |^FAILED|passed|failed" $OUT/pytest.log | cut -c1-400 | head -40
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u tools/diag_mt_nan.py > $OUT/diag.log 2>&1 || true
cut -c1-1500 $OUT/diag.log | tail -12
echo done
