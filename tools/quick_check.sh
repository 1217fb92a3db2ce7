#!/bin/bash
# Quick GPU check of a kernel change: the fit-path parity tests, an optional experiment, the bench
# line (no CPU baseline) and one SQ counter pass over the fit kernels.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py tests/test_gpu_bench_path.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
if [ -n "$EXP" ]; then timeout -k 10 300 python -u $EXP > $OUT/exp.jsonl 2> $OUT/exp.err; cat $OUT/exp.jsonl; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['phases_ms']); print({k: (round(v['avg_us'],1), round(v['avg_us_events'],1)) for k, v in d['roofline']['kernels'].items()})"
if [ -n "$SQ" ]; then
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
fi
echo done
