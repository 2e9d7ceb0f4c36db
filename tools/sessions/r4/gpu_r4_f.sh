#!/bin/bash
# Round-4 session F: parity suite (K-skip final stage, lighter live poll), the
# C-ABI latency probe, the basic-block profile of the product's k_count3c, the
# FIDE PMC passes, rocprofv3 --kernel-trace --stats of the bench, and the bench.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_f.log; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_f.log 2>&1 || { tail -30 $O/pytest_gpu_f.log; exit 1; }
tail -2 $O/pytest_gpu_f.log
step latency
timeout -k 10 60 ./tools/latency_probe 5000 > $O/latency_probe_f.json 2>&1 || { cat $O/latency_probe_f.json; exit 2; }
cat $O/latency_probe_f.json
step bbprof
DCHESS_LIB=$PWD/distributed-chess_amd/build/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7_f.json 4 > $O/bb_f.log 2>&1 || { tail $O/bb_f.log; exit 3; }
step bench
timeout -k 10 400 python -u bench.py > $O/bench_f.json 2> $O/bench_f.err || { tail -20 $O/bench_f.err; exit 4; }
step prof
rm -rf $O/prof_f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_f.json 2> $O/prof_f.err || { tail -20 $O/prof_f.err; exit 5; }
step fidepmc
STAGES=fidepmc bash tools/gpu_round.sh || exit 6
step done
