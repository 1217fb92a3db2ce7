#!/bin/bash
# Persistent k_spec_tile: parity subset, then A/B (FGP_SPEC_PERSIST=1 / 0) of the C4 fit iteration and the C4
# bench line.  Each GPU step has its own limit; a crash or time limit ends the script.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04p}
mkdir -p $OUT
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_spectral.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -15 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
set -e
for rep in 1 2; do
  for P in 1 0; do
    echo "{\"persist\": $P, \"rep\": $rep}" >> $OUT/ab.jsonl
    FGP_SPEC_PERSIST=$P timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 >> $OUT/ab.jsonl 2>> $OUT/ab.err
  done
done
cat $OUT/ab.jsonl
for PG in 00 10 11; do
  FGP_SPEC_PERSIST=${PG:0:1} FGP_SPEC_BASIS_GEN=${PG:1:1} timeout -k 10 300 python -u bench.py --no-secondary --no-multitask --no-paper --no-cpu-baseline > $OUT/bench_$PG.json 2> $OUT/bench_$PG.err
  python -c "import json;d=json.load(open('$OUT/bench_$PG.json'));print('persist,gen=$PG', d['value'], d['ms_per_step'], d.get('phases_ms'), d.get('graph'))"
done
if [ -n "$PERSIST_STAMPS" ]; then timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl; fi
if [ -n "$LIBAB" ]; then
  for v in $LIBAB; do
    FGP_LIB_PATH=fastgaussianprocesses_amd/_lib/exp/libfgp_$v.so timeout -k 10 300 python -u bench.py --no-secondary --no-multitask --no-paper --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err
    python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d.get('phases_ms'))"
  done
fi
if [ -n "$STEPTRACE" ]; then
  timeout -k 10 200 python -u tools/step_trace.py $STEPTRACE > $OUT/step_host_$STEPTRACE.txt 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/st -o t -- python3 tools/step_trace.py $STEPTRACE > /dev/null 2> $OUT/st.err
  python tools/step_trace.py --trace $OUT/st/t_kernel_trace.csv > $OUT/step_trace_$STEPTRACE.txt 2>&1
  head -12 $OUT/step_host_$STEPTRACE.txt; tail -3 $OUT/step_trace_$STEPTRACE.txt
fi
if [ -n "$PROF_SMALL" ]; then timeout -k 10 200 python -u tools/prof_fit_small.py > $OUT/prof_small.txt 2>&1; head -40 $OUT/prof_small.txt; fi
if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
