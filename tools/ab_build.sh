#!/bin/bash
# Builds A/B variants of libdchess.so that differ only in dc_perft.hip's
# compile-time flags (measurement only; tools/ab_perft_time.py times them):
#   tools/ab_build.sh NAME "-DFLAG=1 ..." [NAME2 "FLAGS2" ...]
# -> distributed-chess_amd/build/var/NAME/libdchess.so (the other objects are
# the product build's).  Runs on the CPU host; the .so files travel with gpurun.
set -e
cd "$(dirname "$0")/../distributed-chess_amd"
make -s libdchess.so
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function"
while [ $# -ge 2 ]; do
  N=$1; F=$2; shift 2
  mkdir -p build/var/$N
  ( /opt/rocm/bin/hipcc $HIPFLAGS $F -c csrc/dc_perft.hip -o build/var/$N/dc_perft.o && \
    /opt/rocm/bin/hipcc $HIPFLAGS -shared -o build/var/$N/libdchess.so build/var/$N/dc_perft.o \
      build/dc_moves.o build/dc_hash.o build/dc_txsig.o build/dc_api.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && \
    rm -f build/var/$N/dc_perft.o && echo "built build/var/$N/libdchess.so ($F)" ) &
done
wait
