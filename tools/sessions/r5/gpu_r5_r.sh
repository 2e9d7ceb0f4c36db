#!/bin/bash
# Round-5 session R: where k_count3c's cycles go after the target-side pawn
# correction (basic-block counts of the instrumented build), the child
# categories (A/B build, DC_C2C_PHASE=7), and the FIDE legs after the bench fix.
O=gpurun_out/r5
P=$PWD/distributed-chess_amd
mkdir -p $O
export TMPDIR=/tmp
DCHESS_LIB=$P/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_r.json 4 > $O/bb_r.log 2>&1 || { tail $O/bb_r.log; exit 1; }
DCHESS_LIB=$P/libdchess_ab.so DC_FUSED3=0 DC_C2C_PHASE=7 DEPTH=7 timeout -k 10 120 python -u tools/c2c_stats.py > $O/c2c_stats_r.txt 2>&1 || { tail $O/c2c_stats_r.txt; exit 2; }
cat $O/c2c_stats_r.txt
timeout -k 10 300 python -u bench.py --only fidesuite,fide7 --no-cpu > $O/bench_r.json 2> $O/bench_r.err || { tail -20 $O/bench_r.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/bench_r.json'))
for k in ('fide_perft7','fide_suite_d5'):
    x=d.get(k) or d; print(k, x.get('ms_per_step'), x.get('sequential_ms_per_step'), x.get('final_kernel_ms'), (x.get('roofline') or {}).get('frac'))"
