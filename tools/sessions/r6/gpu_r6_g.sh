#!/bin/bash
# Round 6, session 3: basic-block counts of k_state_hash_ref on the bench's
# workload (tools/bbprof_build.sh hash k_state_hash_ref hash6).
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_hash6/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py hash $O/bb_hash.json > $O/bb_hash.log 2>&1 || { tail -20 $O/bb_hash.log; exit 1; }
tail -3 $O/bb_hash.log
echo done
