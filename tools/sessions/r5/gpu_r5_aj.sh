#!/bin/bash
# Round-5 session AJ: basic-block counts of k_replay_ref4<0,4,true,false> (1M games x 80 plies).
O=gpurun_out/r5
mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_rep/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py replay $O/bb_replay.json 1
