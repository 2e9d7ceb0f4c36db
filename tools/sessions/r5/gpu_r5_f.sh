#!/bin/bash
# Round-5 session F (diagnostics): which co-resident opcode
# corrupts the reproducer's final stage (96 blocks, one per CU), the same
# source without inline-asm shifts as victim, and the shipped kernels beside
# the aggressors.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
nz() { timeout -k 10 300 python -u tools/diag/noise_check.py "$@" >> $O/noise_f.jsonl 2>> $O/noise_f.err; }
DC_DIAG_GRID=96 DCHESS_LIB=$V/t_king_r4_grid/libdchess.so nz --ms 3000 --reps 2 --kinds=1,6,7,8,9,10,11,12,13,14,15 || exit 1
DC_DIAG_GRID=96 DCHESS_LIB=$V/t_king_r4_pad3_grid/libdchess.so nz --ms 3000 --reps 2 --kinds=-1,1,6 || exit 1
nz --ms 3000 --reps 2 --kinds=6,13,14 || exit 1
nz --rules ref --depth 7 --reps 10 --ms 6000 --kinds=6,7,13,14 || exit 1
nz --rules ref --depth 6 --reps 20 --ms 6000 --kinds=1,6 || exit 1
DC_DIAG_GRID=96 DCHESS_LIB=$V/t_king_r4_diag1_grid/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py --noise 1 kiwipete pos6 \
  >> $O/child_diag_f.jsonl 2>> $O/child_diag_f.err || exit 1
DCHESS_LIB=$V/t_king_r4_diag1_grid/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py --noise 1 --noise-blocks 256 kiwipete pos6 \
  >> $O/child_diag_f.jsonl 2>> $O/child_diag_f.err || exit 1
cat $O/noise_f.jsonl
cut -c1-3000 $O/child_diag_f.jsonl
