#!/bin/bash
# Quick GPU iteration: TESTS (pytest -m gpu), then EXP (a python script) -- each with its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  rc=0
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
  tail -15 $OUT/pytest.log
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
fi
if [ -n "$EXP" ]; then
  timeout -k 10 300 python -u $EXP > $OUT/exp.jsonl 2> $OUT/exp.err || { tail -20 $OUT/exp.err; exit 1; }
  cat $OUT/exp.jsonl
fi
echo done
