#!/bin/bash
# Round-5 session E (diagnostics): the round-4 reproducer's
# final stage on 96 blocks (one per CU: exact alone) beside co-resident noise
# waves of one kind each (tools/diag/noise.hip); controls: the product's FIDE
# and REF perft beside the same noise.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
nz() { timeout -k 10 240 python -u tools/diag/noise_check.py "$@" >> $O/noise_e.jsonl 2>> $O/noise_e.err; }
DC_DIAG_GRID=96 DCHESS_LIB=$V/t_king_r4_grid/libdchess.so nz --ms 6000 --kinds=-1,0,1,2,3,4,5 || exit 1
DC_DIAG_GRID=96 DCHESS_LIB=$V/t_king_r4_grid/libdchess.so nz --ms 6000 --kinds 0,1,3 --blocks 256 || exit 1
nz --ms 6000 --kinds=-1,0,1,2 || exit 1
nz --rules ref --depth 7 --reps 10 --ms 8000 --kinds=-1,0,1,2,4 || exit 1
cat $O/noise_e.jsonl
