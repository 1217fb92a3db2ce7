#!/bin/bash
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes of tools/secondary_kernels.py (each pass its
# own run, counters as MI355X_MICROARCH.md prescribes), summarised by tools/secondary_stats.py into $OUT/stats.json.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/secondary}
mkdir -p $OUT
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o t -- python3 tools/secondary_kernels.py --steps 3 > $OUT/trace.log 2>&1
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o p -- python3 tools/secondary_kernels.py --steps 3 > $OUT/pmc_$c.log 2>&1
done
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
F=$(find $OUT/pmc_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find $OUT/pmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
Q=$(find $OUT/pmc_SQ_INSTS_VALU -name "*counter_collection.csv" | head -1)
python3 tools/secondary_stats.py $T --steps 3 --pmc $F $W $Q > $OUT/stats.json
echo done
