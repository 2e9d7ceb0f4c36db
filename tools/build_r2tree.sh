#!/bin/bash
# Rebuilds the round-2 failing tree used by tools/sessions/r3/gpu_r3m.sh and gpu_r3n.sh
# (DESIGN.md section 3.6): commit 3d8df08 in full, its final stage built with
# the struct-of-arrays parents (-DDC_C2C_SOA=1: k_count3c spills 48 B/lane),
# under distributed-chess_amd/build/var/r2tree (git-ignored; travels with gpurun).
set -e
cd "$(dirname "$0")/.."
R=distributed-chess_amd/build/var/r2tree
rm -rf $R && mkdir -p $R
git archive 3d8df08 | tar -x -C $R
rm -rf $R/profiles $R/tests/cpp $R/integration
cp tools/c2c_diag.py tools/c2c_diag_e4.py $R/tools/
make -C $R/distributed-chess_amd -j8 -s libdchess.so \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -DDC_C2C_SOA=1"
echo "built $R/distributed-chess_amd/libdchess.so"
