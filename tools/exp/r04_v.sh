#!/bin/bash
# the LDS-only-barrier patch (tools/exp/r04v_barrier_keep_vm.patch) as an experiment build: parity subset + stamps
# build first (CPU): git apply tools/exp/r04v_barrier_keep_vm.patch && bash tools/build_exp.sh FGP_EXP_KEEPVM=1 keepvm fgp_spectral.hip && git checkout fastgaussianprocesses_amd/csrc/fgp_spectral.hip && python -c "import fastgaussianprocesses_amd.build as b; b.build()"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04v}
mkdir -p $OUT
set -e
export FGP_LIB_PATH=$PWD/fastgaussianprocesses_amd/_lib/exp/libfgp_keepvm.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_bench_path.py -m gpu -q -x --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/exp_persist_stamps.py > $OUT/persist.jsonl 2> $OUT/persist.err
timeout -k 10 120 python -u tools/exp_spec_stamps.py --iters 30 > $OUT/stamps.jsonl 2> $OUT/stamps.err
cut -c1-300 $OUT/persist.jsonl; grep fused $OUT/stamps.jsonl | cut -c1-200
