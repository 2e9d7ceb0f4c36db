#!/bin/bash
# Round-4 session I: parity suite of the product (per-piece knight/king
# enumeration of the special moves), same-box A/B of that change, basic-block profiles of k_count3c and the FIDE final
# stage, the bench, rocprofv3 --kernel-trace --stats of the bench.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_i.log; }
V=distributed-chess_amd/build/var
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_i.log 2>&1 || { tail -30 $O/pytest_gpu_i.log; exit 1; }
tail -2 $O/pytest_gpu_i.log
step ab-piece
timeout -k 10 400 python -u tools/ab_perft_time.py 5 $V/r4_nopiece/libdchess.so $V/r4_piece/libdchess.so > $O/ab_piece_i.jsonl 2>&1 || { tail $O/ab_piece_i.jsonl; exit 3; }
tail -1 $O/ab_piece_i.jsonl
step bbprof
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_i.json 4 > $O/bb_i.log 2>&1 || { tail $O/bb_i.log; exit 5; }
step bench
timeout -k 10 400 python -u bench.py > $O/bench_i.json 2> $O/bench_i.err || { tail -20 $O/bench_i.err; exit 6; }
step prof
rm -rf $O/prof_i
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_i -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_i.json 2> $O/prof_i.err || { tail -20 $O/prof_i.err; exit 7; }
step done
