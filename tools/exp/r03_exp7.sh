#!/bin/bash
# GPU tests (multitask + spectral + bench path + gp), then stamps of the 8-wave tile (default) vs FGP_SPEC_NW=4.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03e7}
mkdir -p $OUT
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_multitask.py tests/test_gpu_spectral.py tests/test_gpu_bench_path.py tests/test_gpu_gp.py -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
grep -E "^E  |^FAILED|passed|failed" $OUT/pytest.log | cut -c1-400 | head -30
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for NW in 8 4; do
  echo "{\"FGP_SPEC_NW\": $NW}" >> $OUT/stamps.jsonl
  FGP_SPEC_NW=$NW timeout -k 10 200 python -u tools/exp_spec_stamps.py --iters 20 >> $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
done
cut -c1-300 $OUT/stamps.jsonl
timeout -k 10 300 python -u tools/paper_kernels.py > $OUT/paper.jsonl 2> $OUT/paper.err || { tail -5 $OUT/paper.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/paper.jsonl'):
    c=json.loads(l); print(c['benchmark'], c['gp'][:12], c['data'], c['iterations'], '%.2e' % c['s_per_step'], c['paper_s_per_step'])
"
echo done
