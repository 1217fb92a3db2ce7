#!/bin/bash
# Round-4 measurement call: the spectral lab, the fit-iteration stamps, smoke, bench (default run) and a
# rocprofv3 kernel-trace of a short bench.  Each GPU step has its own limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04bench}
mkdir -p $OUT
if [ -z "$NOLAB" ]; then timeout -k 10 200 ./tools/spec_lab > $OUT/lab.jsonl 2>&1; cat $OUT/lab.jsonl; fi
timeout -k 10 300 python -u tools/exp_spec_stamps.py > $OUT/stamps.jsonl 2> $OUT/stamps.err
cat $OUT/stamps.jsonl
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_prof.json 2> $OUT/bench_prof.err
echo done
