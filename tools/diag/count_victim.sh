#!/bin/bash
# Builds tools/diag/libcountvictim_<NAME>.so against REV's rule headers:
#   tools/diag/count_victim.sh NAME REV "FLAGS"
set -e
N=$1; REV=$2; F=${3:-}
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
git -C $R archive $REV distributed-chess_amd/csrc include | tar -x -C $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function -I$T/distributed-chess_amd/csrc \
  $F -o $R/tools/diag/libcountvictim_$N.so $R/tools/diag/count_victim.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-function -I$T/distributed-chess_amd/csrc \
  $F --cuda-device-only -S -o $R/distributed-chess_amd/build/asm/r5/countvictim_$N.s $R/tools/diag/count_victim.hip
rm -rf $T
echo "built tools/diag/libcountvictim_$N.so ($REV $F)"
