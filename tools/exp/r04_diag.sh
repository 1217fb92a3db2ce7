#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04diag}
mkdir -p $OUT
timeout -k 10 200 python -u tools/find_syncs.py > $OUT/find_syncs.txt 2>&1; cat $OUT/find_syncs.txt | head -60
timeout -k 10 600 python -u tools/diag_capture.py > $OUT/diag_capture.txt 2>&1; cat $OUT/diag_capture.txt
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl
timeout -k 10 200 python -u tools/step_trace.py C4 > $OUT/step_host_C4.txt 2>&1; head -14 $OUT/step_host_C4.txt
timeout -k 10 200 python -u tools/prof_fit_small.py > $OUT/prof_small.txt 2>&1; head -50 $OUT/prof_small.txt
echo done
