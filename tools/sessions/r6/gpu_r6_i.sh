#!/bin/bash
# Round 6, session 3: the state-hash call's kernel timeline (rocprofv3
# --kernel-trace --stats of bench.py --only hash) and the hash kernel's new
# basic-block counts (tools/bbprof_build.sh hash k_state_hash_ref hash7).
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_hash -o run --output-format csv -- python bench.py --only hash --hash-steps 5 --no-cpu > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_hash7/libdchess_bb.so timeout -k 10 300 python -u tools/bbprof_run.py hash $O/bb_hash.json > $O/bb_hash.log 2>&1 || { tail -20 $O/bb_hash.log; exit 2; }
tail -2 $O/bb_hash.log
echo done
