#!/bin/bash
# Multitask GPU tests + the paper configurations' timings.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03mt2}
mkdir -p $OUT
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_multitask.py -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
grep -E "^E  |^FAILED|passed|failed" $OUT/pytest.log | cut -c1-400 | head -30
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/paper_kernels.py > $OUT/paper.jsonl 2> $OUT/paper.err || { tail -5 $OUT/paper.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/paper.jsonl'):
    c=json.loads(l); print(c['benchmark'], c['gp'][:12], c['data'], c['iterations'], '%.2e' % c['s_per_step'], c['paper_s_per_step'])
"
echo done
