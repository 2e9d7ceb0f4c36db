#!/bin/bash
# One GPU session of the round-4 loop: parity suite of the product, a
# same-box A/B of two library builds, the bench and rocprofv3 --kernel-trace
# --stats of the bench.  Outputs under gpurun_out/r4/ tagged TAG.
#   TAG=k LIB_A=... LIB_B=... [LEGS=ref7] [ROUNDS=5] [SKIP=bench,prof,test] bash tools/gpu_ab_session.sh
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
T=${TAG:?}
step() { echo "[$(date +%T)] $*" >> $O/steps_$T.log; }
skip() { [[ ",${SKIP:-}," == *",$1,"* ]]; }
if ! skip test; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_$T.log 2>&1 || { tail -30 $O/pytest_gpu_$T.log; exit 1; }
  tail -2 $O/pytest_gpu_$T.log
fi
if [ -n "${LIB_A:-}" ]; then
  step ab
  LEGS=${LEGS:-ref7} timeout -k 10 500 python -u tools/ab_perft_time.py ${ROUNDS:-5} $LIB_A $LIB_B > $O/ab_$T.jsonl 2>&1 || { tail $O/ab_$T.jsonl; exit 3; }
  tail -1 $O/ab_$T.jsonl
fi
if ! skip bench; then
  step bench
  timeout -k 10 400 python -u bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { tail -20 $O/bench_$T.err; exit 6; }
fi
if ! skip prof; then
  step prof
  rm -rf $O/prof_$T
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_$T.json 2> $O/prof_$T.err || { tail -20 $O/prof_$T.err; exit 7; }
fi
step done
