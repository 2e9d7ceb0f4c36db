#!/bin/bash
# Round-4 session M: the live validator with two staggered polls in flight --
# its GPU tests, then the C-ABI latency of the old and new wave, alternated.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_m.log; }
V=distributed-chess_amd/build/var
step pytest-live
timeout -k 10 300 python -u -m pytest tests/test_gpu_live.py tests/test_gpu_ref.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_live_m.log 2>&1 || { tail -30 $O/pytest_live_m.log; exit 1; }
tail -2 $O/pytest_live_m.log
for r in 1 2 3; do
  for x in old new; do
    step "latency $x $r"
    timeout -k 10 60 $V/live_$x/tools/latency_probe 5000 > $O/latency_m_${x}_$r.json 2>&1 || { cat $O/latency_m_${x}_$r.json; exit 2; }
    echo "$x $r $(cat $O/latency_m_${x}_$r.json)"
  done
done
step done
