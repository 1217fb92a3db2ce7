#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04h}
mkdir -p $OUT
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_spectral.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
tail -3 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
set -e
timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 > $OUT/stamps.jsonl 2> $OUT/stamps.err; cat $OUT/stamps.jsonl
timeout -k 10 400 python -u bench.py --graph --no-secondary --no-multitask --no-paper --no-cpu-baseline > $OUT/bench_graph.json 2> $OUT/bench_graph.err
python -c "import json;d=json.load(open('$OUT/bench_graph.json'));print('graph', d['value'], d['ms_per_step'], d.get('graph'), d['phases_ms'])"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o sq -- python3 tools/fit_kernels.py > $OUT/pmc_sq.log 2>&1
python3 tools/pmc_sq_summary.py $OUT/pmc_sq/sq_counter_collection.csv > $OUT/pmc_sq.json; python3 -c "
import json;d=json.load(open('$OUT/pmc_sq.json'))
[print(k, v.get('valu_per_wave')) for k,v in d.items() if 'spec_tile' in k]"
if [ $rc -eq 1 ]; then echo "pytest: failures"; exit 1; fi
echo done
