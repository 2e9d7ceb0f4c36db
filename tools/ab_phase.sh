#!/bin/bash
# Timing of k_count2c phases (DC_C2C_PHASE=1/2 give wrong counts: timing only).
export TMPDIR=/tmp
# the knobs below exist only in the A/B build (make -C distributed-chess_amd ab)
export DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so
[ -f "$DCHESS_LIB" ] || { echo "build libdchess_ab.so first (make -C distributed-chess_amd ab)"; exit 3; }
O=gpurun_out; mkdir -p $O
for v in ${AB_VARIANTS:-"DC_C2C_PHASE=0" "DC_C2C_PHASE=1" "DC_C2C_PHASE=2"}; do
  env ${v//,/ } timeout -k 10 120 python -u tools/time_final.py > $O/abp_$v.txt 2> $O/abp_err.log || { cat $O/abp_err.log; exit 2; }
  echo "$v $(cat $O/abp_$v.txt)"
done
