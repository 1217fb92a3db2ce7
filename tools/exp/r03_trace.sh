#!/bin/bash
# Host profile + kernel trace of one step of each config in CFGS (tools/step_trace.py).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}
mkdir -p $OUT
for c in ${CFGS:-C2 C3}; do
  timeout -k 10 200 python -u tools/step_trace.py $c > $OUT/host_$c.txt 2>&1
  head -1 $OUT/host_$c.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_$c -o t -- python3 tools/step_trace.py $c > /dev/null 2>&1
  python tools/step_trace.py --trace $(find $OUT/kt_$c -name "*kernel_trace.csv" | head -1) > $OUT/trace_$c.txt
  tail -1 $OUT/trace_$c.txt
done
echo done
