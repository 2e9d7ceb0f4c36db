#!/bin/bash
# Round-4 session G: parity suite of the product (K-skip, pipelined repeat
# runs, FIDE final stage at 3 blocks/CU, lighter live poll), C-ABI latency,
# A/B of the pipelined repeat and of the FIDE budget, the basic-block profile of
# k_count3c, the bench, rocprofv3 --kernel-trace --stats of the bench, FIDE PMC.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_g.log; }
V=distributed-chess_amd/build/var
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_g.log 2>&1 || { tail -30 $O/pytest_gpu_g.log; exit 1; }
tail -2 $O/pytest_gpu_g.log
step latency
timeout -k 10 60 ./tools/latency_probe 5000 > $O/latency_probe_g.json 2>&1 || { cat $O/latency_probe_g.json; exit 2; }
cat $O/latency_probe_g.json
step ab-pipe
LEGS=ref7 timeout -k 10 300 python -u tools/ab_perft_time.py 5 $V/r4_nopipe/libdchess.so $V/r4_pipe/libdchess.so > $O/ab_pipe_g.jsonl 2>&1 || { tail $O/ab_pipe_g.jsonl; exit 3; }
tail -1 $O/ab_pipe_g.jsonl
step ab-fide
LEGS=fide7,suite timeout -k 10 300 python -u tools/ab_perft_time.py 3 $V/r4_fide4/libdchess.so $V/r4_cur/libdchess.so > $O/ab_fide_g.jsonl 2>&1 || { tail $O/ab_fide_g.jsonl; exit 4; }
tail -1 $O/ab_fide_g.jsonl
step bbprof
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_g.json 4 > $O/bb_g.log 2>&1 || { tail $O/bb_g.log; exit 5; }
step bench
timeout -k 10 400 python -u bench.py > $O/bench_g.json 2> $O/bench_g.err || { tail -20 $O/bench_g.err; exit 6; }
step prof
rm -rf $O/prof_g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_g -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_g.json 2> $O/prof_g.err || { tail -20 $O/prof_g.err; exit 7; }
step fidepmc
STAGES=fidepmc bash tools/gpu_round.sh || exit 8
step done
