#!/bin/bash
# Round-5 session S: basic-block counts of k_count3c<0,...> (perft(7)) after the
# target-side pawn correction.
O=gpurun_out/r5
P=$PWD/distributed-chess_amd
mkdir -p $O
export TMPDIR=/tmp
DCHESS_LIB=$P/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_s.json 4 > $O/bb_s.log 2>&1 || { tail $O/bb_s.log; exit 1; }
tail -2 $O/bb_s.log
