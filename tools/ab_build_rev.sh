#!/bin/bash
# A/B baseline from a git revision: dc_perft.hip (and the headers it
# includes) as of REV (WT: the working tree), linked with the working tree's
# other objects (measurement only; tools/ab_perft_time.py times the libraries).
#   [SRCS="dc_perft dc_api"] [PATCH="cmd"] tools/ab_build_rev.sh NAME REV ["FLAGS"]
# (SRCS: the sources taken from REV, default dc_perft)
# -> distributed-chess_amd/build/var/NAME/libdchess.so
set -e
N=$1; REV=$2; F=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
if [ "$REV" = WT ]; then
  (cd $R && tar -c distributed-chess_amd/csrc include) | tar -x -C $T
else
  git -C $R archive $REV distributed-chess_amd/csrc include | tar -x -C $T
fi
# PATCH: a command run in the exported tree before building (diagnostics)
if [ -n "${PATCH:-}" ]; then (cd $T && eval "$PATCH"); fi
cd $R/distributed-chess_amd
make -s libdchess.so
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -I$T/include"
mkdir -p build/var/$N
OBJS=""
for u in dc_perft dc_moves dc_hash dc_txsig dc_api; do
  if [[ " ${SRCS:-dc_perft} " == *" $u "* ]]; then
    /opt/rocm/bin/hipcc $HIPFLAGS $F -c $T/distributed-chess_amd/csrc/$u.hip -o build/var/$N/$u.o
    OBJS="$OBJS build/var/$N/$u.o"
  else
    OBJS="$OBJS build/$u.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/var/$N/libdchess.so $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f build/var/$N/*.o
rm -rf $T
echo "built build/var/$N/libdchess.so (${SRCS:-dc_perft} at $REV $F)"
