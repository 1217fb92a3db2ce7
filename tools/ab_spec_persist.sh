#!/bin/bash
# A/B of the launch-per-iteration k_spec_tile against its persistent instance (FGP_SPEC_PERSIST=1) on the C4 bench
# step, after the 32-bit DMA offsets; plus the spectral / bench-path / C5 GPU tests.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dma}
mkdir -p $OUT
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_multioutput.py > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
B="--no-cpu-baseline --no-secondary --no-multitask --no-paper"
timeout -k 10 200 python bench.py $B --steps 5 > $OUT/bench_default.json 2> $OUT/b1.err
FGP_SPEC_PERSIST=1 timeout -k 10 200 python bench.py $B --steps 5 > $OUT/bench_persist.json 2> $OUT/b2.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pd -o p -- python3 bench.py --steps 2 --warmup 1 $B --no-graph > $OUT/pd.log 2>&1
FGP_SPEC_PERSIST=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pp -o p -- python3 bench.py --steps 2 --warmup 1 $B --no-graph > $OUT/pp.log 2>&1
echo done
