#!/bin/bash
# Round-4 session S: the deep FIDE published counts on the GPU, then the
# product's bench, rocprofv3 --kernel-trace --stats of it, and the PMC passes
# (REF legs, then FIDE legs) that feed profiles/pmc_latest.json.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
echo "[$(date +%T)] fide-deep" >> $O/steps_s.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fide.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_fide_s.log 2>&1 || { tail -30 $O/pytest_fide_s.log; exit 1; }
tail -2 $O/pytest_fide_s.log
echo "[$(date +%T)] bench+prof+pmc" >> $O/steps_s.log
STAGES="bench prof pmc fidepmc" bash tools/gpu_round.sh || exit $?
