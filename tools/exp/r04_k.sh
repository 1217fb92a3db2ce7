#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04k}
mkdir -p $OUT
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_gp.py tests/test_gpu_multitask.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -3 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
set -e
timeout -k 10 400 python -u bench.py --no-secondary --no-multitask --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "
import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'])
[print(c['benchmark'], c['gp'][:6], c['data'], round(c['s_per_step']*1e6,1)) for c in d['paper']['configs']]"
if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
