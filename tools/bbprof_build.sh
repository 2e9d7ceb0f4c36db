#!/bin/bash
# Build an instrumented copy of the product library: ONE kernel's device
# assembly instrumented by tools/bbprof.py (basic-block execution counts per wave).
#   tools/bbprof_build.sh perft|moves KERNEL_SUBSTR TAG
# Output: distributed-chess_amd/build/bb_TAG/libdchess_bb.so and the
# uninstrumented assembly build/bbtmp_FILE/dc_FILE-orig.s (same block numbering).
# The device compile (hipcc -save-temps, -DDC_BBPROF) is kept in
# build/bbtmp_FILE and reused while its source is older than it.
# Measurement only: nothing in the product, tests or bench loads these
# libraries unless DCHESS_LIB points at one (tools/bbprof_run.py).
set -e
FILE=$1
KSUB=$2
TAG=$3
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/distributed-chess_amd
T=$P/build/bbtmp_$FILE
B=$P/build/bb_$TAG
SRC=$P/csrc/dc_$FILE.hip
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -DDC_BBPROF"
DEV=dc_$FILE-hip-amdgcn-amd-amdhsa-gfx950.s
make -s -C $P libdchess.so > /dev/null
stale=0
[ -f $T/dc_$FILE-orig.s ] || stale=1
for h in $SRC $P/csrc/*.h $R/include/dchess.h; do [ $stale = 1 ] || [ $h -nt $T/dc_$FILE-orig.s ] && stale=1; done
if [ $stale = 1 ]; then
  rm -rf $T && mkdir -p $T && cd $T
  /opt/rocm/bin/hipcc -### -save-temps $FLAGS -c $SRC -o $T/dc_$FILE.o 2> cmds.txt
  /opt/rocm/bin/hipcc -save-temps $FLAGS -c $SRC -o $T/dc_$FILE.o 2> /dev/null
  cp $DEV dc_$FILE-orig.s
fi
rm -rf $B && cp -r $T $B && cd $B
python3 $R/tools/bbprof.py instrument dc_$FILE-orig.s $DEV --kernel "$KSUB" --sym dc_bbprof_$FILE
# re-run the pipeline from the device assembler on (cc1as, lld, bundler, host)
python3 - "$B" "$T" <<'PY'
import shlex, subprocess, sys
b, t = sys.argv[1], sys.argv[2]
cmds = [shlex.split(l) for l in open(b + "/cmds.txt") if l.startswith(' "')]
i = next(k for k, c in enumerate(cmds) if "-cc1as" in c and "amdgcn-amd-amdhsa" in c)
for c in cmds[i:]:
    c = [x.replace(t, b) for x in c]
    subprocess.check_call(c, cwd=b, stderr=subprocess.DEVNULL)
PY
OBJS=""
for f in moves perft hash txsig api; do
  if [ $f = $FILE ]; then OBJS="$OBJS $B/dc_$f.o"; else OBJS="$OBJS $P/build/dc_$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o $B/libdchess_bb.so $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
# keep only what a GPU run loads
find $B -type f ! -name libdchess_bb.so ! -name "*.json" -delete
echo "built $B/libdchess_bb.so"
