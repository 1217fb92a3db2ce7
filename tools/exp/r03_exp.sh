#!/bin/bash
# Round-3 experiment call: EXP (a python script with args) plain, then under rocprofv3 --kernel-trace --stats.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-exp}
mkdir -p $OUT
timeout -k 10 300 python -u $EXP > $OUT/exp.jsonl 2> $OUT/exp.err || { tail -20 $OUT/exp.err; exit 1; }
cat $OUT/exp.jsonl
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o exp -- python3 -u $EXP > $OUT/exp_prof.jsonl 2> $OUT/exp_prof.err || { tail -5 $OUT/exp_prof.err; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 tools/kstats.py {} 2>/dev/null | head -25 || true
fi
echo done
