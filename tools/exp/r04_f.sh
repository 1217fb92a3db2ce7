#!/bin/bash
# the bench lines (with and without --graph), the rocprofv3 kernel trace of a short bench, PMC passes of the fit
# kernels.  Each GPU step has its own limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04f}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --graph --no-multitask --no-paper --no-cpu-baseline > $OUT/bench_graph.json 2> $OUT/bench_graph.err
python -c "import json;d=json.load(open('$OUT/bench_graph.json'));print('graph', d['value'], d['ms_per_step'], d.get('graph'));[print(s['config']['workload'][:30], round(s['ms_per_step'],3), s.get('graph')) for s in d.get('secondary') or []]"
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  python -c "import json;d=json.load(open('$OUT/bench.json'));print('eager', d['value'], d['ms_per_step'], d['phases_ms'])"
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-multitask --no-paper > $OUT/bench_prof.json 2> $OUT/bench_prof.err
python tools/kstats_grid.py $OUT/prof/bench_kernel_trace.csv 40 > $OUT/grid_stats.txt; head -12 $OUT/grid_stats.txt
if [ -n "$PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 tools/fit_kernels.py > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 tools/fit_kernels.py > $OUT/pmc_write.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
fi
echo done
