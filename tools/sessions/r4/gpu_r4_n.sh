#!/bin/bash
# Round-4 session N: basic-block profile of k_count3c (special-only slider
# targets), then parity + same-box A/B of the merged pawn-push enumeration.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
echo "[$(date +%T)] bbprof" >> $O/steps_n.log
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_n.json 4 > $O/bb_n.log 2>&1 || { tail $O/bb_n.log; exit 5; }
TAG=n LIB_A=distributed-chess_amd/build/var/r4_stgt/libdchess.so LIB_B=distributed-chess_amd/build/var/r4_push/libdchess.so ROUNDS=6 SKIP=prof,bench bash tools/gpu_ab_session.sh
