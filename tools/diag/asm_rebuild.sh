#!/bin/bash
# Rebuild a diagnostic library whose dc_perft device assembly went through an
# edit (DESIGN.md §3.6 fault study): same compile pipeline as hipcc
# (-save-temps), with tools/diag/asm_edit.py applied to the device .s before
# it is assembled, linked, bundled and embedded in the host object.
#   tools/diag/asm_rebuild.sh NAME REV "FLAGS" "EDIT ARGS"
# REV's dc_perft.hip + dc_api.hip (tools/diag/grid_patch.py applied), the
# working tree's other objects -> distributed-chess_amd/build/var/NAME/libdchess.so
set -e
N=$1; REV=$2; F=$3; E=$4
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
git -C $R archive $REV distributed-chess_amd/csrc include | tar -x -C $T
python $R/tools/diag/grid_patch.py $T/distributed-chess_amd/csrc/dc_perft.hip
cd $T/distributed-chess_amd
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -I$T/include"
/opt/rocm/bin/hipcc -v $HF $F -save-temps -c csrc/dc_perft.hip -o dc_perft.o 2> cmds.log >/dev/null
grep -E '^\s*"/opt' cmds.log > cmds.txt
[ "$(wc -l < cmds.txt)" = 10 ] || { echo "unexpected pipeline"; exit 1; }
python $R/tools/diag/asm_edit.py dc_perft-hip-amdgcn-amd-amdhsa-gfx950.s $E
for i in 4 5 6 8 9 10; do eval "$(sed -n ${i}p cmds.txt)" > /dev/null 2>&1 || { echo "step $i failed"; exit 1; }; done
/opt/rocm/bin/hipcc $HF -c csrc/dc_api.hip -o dc_api.o 2>/dev/null
mkdir -p $R/distributed-chess_amd/build/var/$N
B=$R/distributed-chess_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $B/var/$N/libdchess.so dc_perft.o dc_api.o $B/dc_moves.o $B/dc_hash.o \
  $B/dc_txsig.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
cp dc_perft-hip-amdgcn-amd-amdhsa-gfx950.s $B/var/$N/device.s
rm -rf $T
echo "built build/var/$N/libdchess.so ($REV $F; edit: $E)"
