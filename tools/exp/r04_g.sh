#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04g}
mkdir -p $OUT
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread -k "single_launch or persistent" > $OUT/pytest.log 2>&1 || rc=$?
tail -4 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err; cat $OUT/persist.jsonl
bash tools/r04_f.sh
