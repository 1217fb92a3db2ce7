#!/bin/bash
# Round-3 verification of the committed tree: the whole -m gpu suite, smoke, the bench line (CPU baseline
# included), the rocprofv3 kernel-trace summary of the bench command, PMC passes (FETCH / WRITE / SQ) of
# the fit kernels, the kernel trace of the paper configurations.  Every GPU step has its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03f}
mkdir -p $OUT
TAG=${TAG:-r03f} bash tools/r03_round.sh
TAG=${TAG:-r03f}/pmc DRV=tools/fit_kernels.py bash tools/r03_pmc.sh > $OUT/pmc.txt 2>&1 || { tail -5 $OUT/pmc.txt; exit 1; }
tail -4 $OUT/pmc.txt
find $OUT/pmc -name "*.csv" -size +2M -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ptrace -o paper -- python3 tools/paper_kernels.py > $OUT/paper.jsonl 2> $OUT/paper.err || { tail -5 $OUT/paper.err; exit 1; }
cp $(find $OUT/ptrace -name "*kernel_stats.csv" | head -1) $OUT/paper_kernel_stats.csv
python3 tools/kstats_grid.py $(find $OUT/ptrace -name "*kernel_trace.csv" | head -1) 25 > $OUT/paper_kernel_grid_stats.txt
rm -rf $OUT/ptrace
head -12 $OUT/paper_kernel_grid_stats.txt
echo done
