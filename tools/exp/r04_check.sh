#!/bin/bash
# Round-4 GPU check: the -m gpu suite (or a subset: TESTS=...), then (LAB=1) the spectral lab.  Each GPU step
# has its own limit; a crash / abort / time limit ends the script (no further GPU step).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04chk}
mkdir -p $OUT
prc=0
if [ -z "$NOTESTS" ]; then
  timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=8 --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || prc=$?
  tail -40 $OUT/pytest_gpu.log
  if [ $prc -gt 1 ]; then echo "pytest rc=$prc"; exit $prc; fi
fi
if [ -n "$LAB" ]; then
  timeout -k 10 200 ./tools/spec_lab > $OUT/lab.jsonl 2>&1; rc=$?
  cat $OUT/lab.jsonl
  if [ $rc -ne 0 ]; then echo "lab rc=$rc"; exit $rc; fi
fi
if [ $prc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
