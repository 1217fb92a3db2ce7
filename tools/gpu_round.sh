#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprofv3 kernel stats (+ PMC passes with PMC=1).
# Every GPU step has its own time limit; the script stops at the first crash or timeout.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
if [ -n "$DIAG" ]; then timeout -k 10 300 python -u $DIAG > $OUT/diag.log 2>&1; fi
if [ -z "$NOTEST" ]; then
  rc=0
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
  tail -3 $OUT/pytest_gpu.log
  # stop on a crash/timeout of the test process (not on ordinary test failures, rc=1)
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
timeout -k 10 400 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_prof.json 2> $OUT/bench_prof.err
if [ -n "$PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 tools/fit_kernels.py > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 tools/fit_kernels.py > $OUT/pmc_write.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
fi
echo done
