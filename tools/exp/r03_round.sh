#!/bin/bash
# Round-3 full GPU check: the whole -m gpu suite, smoke, the bench line (with the CPU baseline), and the
# rocprofv3 --kernel-trace --stats summary of the bench command.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03round}
mkdir -p $OUT
rc=0
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
tail -6 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['phases_ms']); print({k: (round(v['avg_us'],1), round(v['avg_us_events'],1)) for k, v in d['roofline']['kernels'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_prof.json 2> $OUT/bench_prof.err
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp $KS $OUT/bench_kernel_stats.csv
KT=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kstats_grid.py $KT > $OUT/bench_kernel_grid_stats.txt 2>/dev/null || true
rm -rf $OUT/prof          # raw traces stay on the box (gpurun_out is copied back only under 64 MiB)
python3 tools/kstats.py $OUT/bench_kernel_stats.csv 20
echo done
