#!/bin/bash
# A/B of experiment builds (tools/build_exp.sh) on the C4 fit iteration: exp_spec_stamps.py per library,
# interleaved, each with its own time limit.  VARIANTS="name ..." (default: the in-tree build and every exp lib).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04ab}
mkdir -p $OUT
L=fastgaussianprocesses_amd/_lib
for rep in 1 2; do
  for v in ${VARIANTS:-hip $(ls $L/exp/ | sed -n 's/^libfgp_\(.*\)\.so$/\1/p')}; do
    if [ "$v" = hip ]; then lib=$L/libfgp_hip.so; else lib=$L/exp/libfgp_$v.so; fi
    echo "{\"build\": \"$v\", \"rep\": $rep}" >> $OUT/ab.jsonl
    FGP_LIB_PATH=$lib timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 >> $OUT/ab.jsonl 2>> $OUT/ab.err
  done
done
cat $OUT/ab.jsonl
if [ -n "$PROF_SMALL" ]; then timeout -k 10 200 python -u tools/prof_fit_small.py > $OUT/prof_small.txt 2>&1; head -80 $OUT/prof_small.txt; fi
if [ -n "$PERSIST" ]; then timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl; fi
if [ -n "$STEPTRACE" ]; then
  timeout -k 10 200 python -u tools/step_trace.py $STEPTRACE > $OUT/step_host_$STEPTRACE.txt 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/st -o t -- python3 tools/step_trace.py $STEPTRACE > /dev/null 2> $OUT/st.err
  python tools/step_trace.py --trace $OUT/st/t_kernel_trace.csv > $OUT/step_trace_$STEPTRACE.txt 2>&1
  head -60 $OUT/step_host_$STEPTRACE.txt; head -80 $OUT/step_trace_$STEPTRACE.txt
fi
