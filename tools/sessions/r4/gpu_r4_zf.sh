#!/bin/bash
# Round 4, session ZF: the live validator's n = 1 REF validate from
# cross-lane ballots (DC_LIVE_GATHER=1, product) -- live-path tests, then the
# product alternated with the one-lane board assembly (DC_LIVE_GATHER=0).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_live.py -x -v --timeout 120 --timeout-method thread > $O/pytest_live_zf.log 2>&1 || { tail -30 $O/pytest_live_zf.log; exit 1; }
tail -2 $O/pytest_live_zf.log
V=distributed-chess_amd/build/var/live0
: > $O/live_gather_zf.txt
for r in 1 2 3; do
  echo "gather $(timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_gather_zf.txt || exit 2
  echo "assemble $(LD_LIBRARY_PATH=$V timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_gather_zf.txt || exit 3
done
cat $O/live_gather_zf.txt
