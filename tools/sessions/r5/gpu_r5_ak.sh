#!/bin/bash
# Round-5 session AK: basic-block counts of the shipped k_count3c<0,4592,4,u32> (perft(7)).
O=gpurun_out/r5
mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py perft7 $O/bb_c3c.json 4
