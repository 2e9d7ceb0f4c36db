#!/bin/bash
# Round-4 session H: parity suite of the product (attack/line tables, no
# pipelined repeat), same-box A/B of the tables (REF perft(7), FIDE legs) and
# of the FIDE budget, basic-block profiles of k_count3c and the FIDE final
# stage, the bench, rocprofv3 --kernel-trace --stats of the bench.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_h.log; }
V=distributed-chess_amd/build/var
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_h.log 2>&1 || { tail -30 $O/pytest_gpu_h.log; exit 1; }
tail -2 $O/pytest_gpu_h.log
step ab-tab
timeout -k 10 400 python -u tools/ab_perft_time.py 5 $V/r4_notab/libdchess.so $V/r4_tab/libdchess.so > $O/ab_tab_h.jsonl 2>&1 || { tail $O/ab_tab_h.jsonl; exit 3; }
tail -1 $O/ab_tab_h.jsonl
step ab-fide
LEGS=fide7,suite timeout -k 10 300 python -u tools/ab_perft_time.py 3 $V/r4_fide4/libdchess.so $V/r4_tab/libdchess.so > $O/ab_fide_h.jsonl 2>&1 || { tail $O/ab_fide_h.jsonl; exit 4; }
tail -1 $O/ab_fide_h.jsonl
step bbprof
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_h.json 4 > $O/bb_h.log 2>&1 || { tail $O/bb_h.log; exit 5; }
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_fide/libdchess_bb.so timeout -k 10 180 python -u tools/bbprof_run.py fide7 $O/bb_fide7_h.json 2 >> $O/bb_h.log 2>&1 || { tail $O/bb_h.log; exit 5; }
step bench
timeout -k 10 400 python -u bench.py > $O/bench_h.json 2> $O/bench_h.err || { tail -20 $O/bench_h.err; exit 6; }
step prof
rm -rf $O/prof_h
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_h -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_h.json 2> $O/prof_h.err || { tail -20 $O/prof_h.err; exit 7; }
step done
