#!/bin/bash
# Round-5 session AG: basic-block counts of k_gen_games_ref (1M games x 80 plies).
O=gpurun_out/r5
mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_gen/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py gen $O/bb_gen.json 1
