#!/bin/bash
# Experiment builds of the real-even kernels: fgp_nll_re.hip compiled with -D$1, linked with the other
# objects of the in-tree build into fastgaussianprocesses_amd/_lib/exp/libfgp_$2.so (select with
# FGP_LIB_PATH).  Timing-only variants: their results are not meant to be correct.
set -e
cd "$(dirname "$0")/.."
L=fastgaussianprocesses_amd/_lib
mkdir -p $L/exp
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC -D$1 -c fastgaussianprocesses_amd/csrc/fgp_nll_re.hip -o $L/exp/re_$2.o
objs=$(ls $L/obj/*.o | grep -v fgp_nll_re.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/exp/libfgp_$2.so $objs $L/exp/re_$2.o
echo built $L/exp/libfgp_$2.so
