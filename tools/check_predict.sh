#!/bin/bash
# k_post_mean change check: the posterior GPU tests, the bench line (C4 + secondaries), the bench command's
# timed-region kernel trace, the predict kernels' trace
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pm}
mkdir -p $OUT
set -e
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_gp.py tests/test_gpu_multioutput.py tests/test_gpu_bench_path.py tests/test_gpu_single_extras.py > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
B="--no-cpu-baseline --no-multitask --no-paper"
timeout -k 10 400 python bench.py $B > $OUT/bench.json 2> $OUT/b.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o p -- python3 bench.py --steps 5 --warmup 1 $B --no-secondary > $OUT/prof.log 2>&1
python tools/timed_region_stats.py $OUT/prof/p_kernel_trace.csv 8 > $OUT/timed_stats.txt; head -5 $OUT/timed_stats.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/ptrace -o trace -- python3 tools/predict_kernels.py > $OUT/ptrace.log 2>&1
python tools/kstats_grid.py $OUT/ptrace/trace_kernel_trace.csv 12 > $OUT/predict_grid_stats.txt; grep post_mean $OUT/predict_grid_stats.txt
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['phases_ms']['post_mean']);[print(s['config'].get('workload','')[:24],s.get('graph',{}).get('phases_ms')) for s in d['secondary']]"
