#!/bin/bash
# Builds diagnostic variants of libdchess.so for the c2c_group investigation
#  into distributed-chess_amd/build/var/:
#   soa      -DDC_C2C_SOA=1                     (the round-2 failing layout, 4 waves/SIMD)
#   soa_st   -DDC_C2C_SOA=1 -DDC_C3C_STATIC=1   (same, static group order: no counter)
#   aos_st   -DDC_C3C_STATIC=1                  (control: shipped layout, static order)
#   soa_pad1/2/3  the soa build with the 64-bit shift statements padded (dc_bits.h DC_SHIFT_PAD)
# Extra -D flags for every variant: EXTRA="-DFOO=1" tools/c2c_variants.sh
# Run on the CPU host (hipcc cross-compiles); the .so files travel with gpurun.
set -e
cd "$(dirname "$0")/../distributed-chess_amd"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function"
SRCS="csrc/dc_moves.hip csrc/dc_perft.hip csrc/dc_hash.hip csrc/dc_txsig.hip csrc/dc_api.hip"
VARIANTS=${VARIANTS:-"soa soa_st aos_st"}
mkdir -p build/var
flags_of() {
  case $1 in
    soa) echo "-DDC_C2C_SOA=1" ;;
    soa_st) echo "-DDC_C2C_SOA=1 -DDC_C3C_STATIC=1" ;;
    aos_st) echo "-DDC_C3C_STATIC=1" ;;
    soa_pad1) echo "-DDC_C2C_SOA=1 -DDC_SHIFT_PAD=1" ;;   # s_nop 1 ahead of every asm 64-bit shift
    soa_pad2) echo "-DDC_C2C_SOA=1 -DDC_SHIFT_PAD=2" ;;   # s_nop 1 after it
    soa_pad3) echo "-DDC_C2C_SOA=1 -DDC_SHIFT_PAD=3" ;;   # plain C shifts
    soa_log) echo "-DDC_C2C_SOA=1 -DDC_C3C_LOG=1" ;;      # + per-group histogram log (dc_ab_c3c_log)
    aos_log) echo "-DDC_C3C_LOG=1" ;;
    rec) echo "-DDC_C2C_REC=1" ;;                          # 48-byte parent records (one LDS address per thread)
    soa_otid) echo "-DDC_C2C_REC=0 -DDC_C2C_SOA=1" ;;      # the soa layout built from the spill-free (otid) source
    soa_r2) echo "-DDC_C2C_SOA=1" ;;                       # round 2's failing build, rebuilt from commit 3d8df08
    nodq) echo "-DDC_C2C_DIAGQ=0" ;;                       # round-3 v2 final stage: every non-quiet child recounted in full
    *) echo "unknown variant $1" >&2; exit 1 ;;
  esac
}
for v in $VARIANTS; do
  F="$(flags_of $v) $EXTRA"
  mkdir -p build/var/$v
  SRC=csrc/dc_perft.hip
  if [ $v = soa_r2 ]; then
    # round 2's failing final stage exactly: dc_perft.hip and its headers as of
    # commit 3d8df08 (thread index live across c2c_group, 44-52 B/lane of
    # spills) with the struct-of-arrays parents
    rm -rf build/var/soa_r2/src && mkdir -p build/var/soa_r2/src
    git -C .. archive 3d8df08 distributed-chess_amd/csrc include | tar -x -C build/var/soa_r2/src
    SRC=build/var/soa_r2/src/distributed-chess_amd/csrc/dc_perft.hip
  fi
  # only dc_perft.hip depends on these flags; the rest are shared objects of the product build
  /opt/rocm/bin/hipcc $HIPFLAGS $F -c $SRC -o build/var/$v/dc_perft.o &
done
wait
for v in $VARIANTS; do
  /opt/rocm/bin/hipcc $HIPFLAGS -shared -o build/var/lib_$v.so build/var/$v/dc_perft.o \
    build/dc_moves.o build/dc_hash.o build/dc_txsig.o build/dc_api.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build/var/lib_$v.so ($(flags_of $v) $EXTRA)"
done
