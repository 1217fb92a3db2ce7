#!/bin/bash
# One GPU call of a round's check: the whole -m gpu suite, smoke, the default bench line, a rocprofv3 kernel trace
# of the bench, PMC passes of the fit kernels (tools/fit_kernels.py) and of the prediction kernels
# (tools/predict_kernels.py: SQ pass + kernel trace).  Each GPU step has its own limit; a crash ends the script.
#   TAG=r05a [NOTESTS=1] [NOBENCH=1] [NOPMC=1] [TESTS="tests/test_x.py ..."] bash tools/final_check.sh
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
rc=0
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
  tail -15 $OUT/pytest_gpu.log
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
fi
set -e
if [ -z "$NOBENCH" ]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['roofline_predict'].get('frac'))"
  # the bench command itself (graph replays in its timed region): every launch, and the timed region's alone
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-multitask --no-paper > $OUT/bench_prof.json 2> $OUT/bench_prof.err
  python tools/kstats_grid.py $OUT/prof/bench_kernel_trace.csv 60 > $OUT/grid_stats.txt; head -8 $OUT/grid_stats.txt
  python tools/timed_region_stats.py $OUT/prof/bench_kernel_trace.csv 60 > $OUT/timed_stats.txt; head -6 $OUT/timed_stats.txt; tail -1 $OUT/timed_stats.txt
fi
if [ -z "$NOPMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 tools/fit_kernels.py > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 tools/fit_kernels.py > $OUT/pmc_write.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmcp_sq -o sq -- python3 tools/predict_kernels.py > $OUT/pmcp_sq.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ptrace -o trace -- python3 tools/predict_kernels.py > $OUT/ptrace.log 2>&1
  python tools/kstats_grid.py $OUT/ptrace/trace_kernel_trace.csv 40 > $OUT/predict_grid_stats.txt
fi
if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
