#!/bin/bash
# single-workgroup persistent reduce: parity (persistent vs launch-per-iteration, spectral tests) + stamps
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04t}
mkdir -p $OUT
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_gp.py -m gpu -q -x --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err
cut -c1-330 $OUT/persist.jsonl
