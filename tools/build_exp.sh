#!/bin/bash
# Experiment builds: the sources named after the first two arguments (default fgp_nll_re.hip) compiled
# with -D for every word of $1 (e.g. "FGP_SPEC_RING=3 FGP_SPEC_PRE=3"), linked with the other objects of the in-tree build into
# fastgaussianprocesses_amd/_lib/exp/libfgp_$2.so (select with FGP_LIB_PATH).  Timing-only variants.
set -e
cd "$(dirname "$0")/.."
L=fastgaussianprocesses_amd/_lib
mkdir -p $L/exp
DEF=$1; NAME=$2; shift 2
SRCS=${@:-fgp_nll_re.hip}
objs=$(ls $L/obj/*.o)
pids=""
for S in $SRCS; do
  o=$L/exp/${NAME}_${S%.hip}.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC $(for w in $DEF; do echo -D$w; done) -c fastgaussianprocesses_amd/csrc/$S -o $o &
  pids="$pids $!"
  objs=$(echo "$objs" | grep -v "/${S%.hip}.o")
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/exp/libfgp_$NAME.so $objs $(for S in $SRCS; do echo $L/exp/${NAME}_${S%.hip}.o; done)
echo built $L/exp/libfgp_$NAME.so
