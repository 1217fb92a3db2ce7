#!/bin/bash
# k_spec_tile change check: the spectral / bench-path / fit GPU tests, the C4 bench line, a kernel trace of the bench
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-spec}
mkdir -p $OUT
set -e
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_gp.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
B="--no-cpu-baseline --no-secondary --no-multitask --no-paper"
timeout -k 10 200 python bench.py $B --steps 10 > $OUT/bench.json 2> $OUT/b.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --steps 2 --warmup 1 $B --no-graph > $OUT/prof.log 2>&1
python tools/kstats_grid.py $OUT/prof/p_kernel_trace.csv 12 > $OUT/grid_stats.txt; head -6 $OUT/grid_stats.txt
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['phases_ms']['fit'],d['roofline'].get('avg_us_device_clock'),d['roofline'].get('avg_us_events'))"
