#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04p2}
mkdir -p $OUT
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_gp.py tests/test_gpu_multioutput.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -4 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "^FAILED|Error" $OUT/pytest.log | head -10; exit $rc; fi
set -e
timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 > $OUT/stamps.jsonl 2> $OUT/stamps.err; cat $OUT/stamps.jsonl
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl
echo done
