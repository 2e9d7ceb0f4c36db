#!/bin/bash
# Round-5 session AF: basic-block counts of k_state_hash_ref (bench workload).
O=gpurun_out/r5
mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_hash/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py hash $O/bb_hash.json 1
