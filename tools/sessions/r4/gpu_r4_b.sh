#!/bin/bash
# Round-4 session B: basic-block profiles of the three hot kernels
# (tools/bbprof_build.sh libraries) and the C-ABI latency probe.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_b.log; }
P=$PWD/distributed-chess_amd/build
step bb-c3c
DCHESS_LIB=$P/bb_c3c/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bb_c3c_d7.json 4 > $O/bb.log 2>&1 || { tail $O/bb.log; exit 1; }
step bb-replay
DCHESS_LIB=$P/bb_replay/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py replay $O/bb_replay.json 2 >> $O/bb.log 2>&1 || { tail $O/bb.log; exit 2; }
step bb-gen
DCHESS_LIB=$P/bb_gen/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py gen $O/bb_gen.json 2 >> $O/bb.log 2>&1 || { tail $O/bb.log; exit 3; }
cat $O/bb.log
step latency
timeout -k 10 60 ./tools/latency_probe 5000 > $O/latency_probe.json 2>&1 || { cat $O/latency_probe.json; exit 4; }
cat $O/latency_probe.json
step tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_live.py tests/test_spill_free.py -x -v --timeout 120 --timeout-method thread > $O/pytest_live_b.log 2>&1 || { tail -30 $O/pytest_live_b.log; exit 5; }
tail -3 $O/pytest_live_b.log
step done
