#!/bin/bash
# Round-4 GPU check: (optional) the spectral lab, then the -m gpu suite (or a subset: TESTS=...).  Each GPU step
# has its own limit; a crash / abort / time limit ends the script (no further GPU step).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04chk}
mkdir -p $OUT
if [ -n "$LAB" ]; then
  timeout -k 10 200 ./tools/spec_lab > $OUT/lab.jsonl 2>&1; rc=$?
  cat $OUT/lab.jsonl
  if [ $rc -ne 0 ]; then echo "lab rc=$rc"; exit $rc; fi
fi
if [ -z "$NOTESTS" ]; then
  rc=0
  timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
  tail -25 $OUT/pytest_gpu.log
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
  if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
fi
echo done
