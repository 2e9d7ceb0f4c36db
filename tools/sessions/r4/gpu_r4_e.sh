#!/bin/bash
# Round-4 session E: GPU parity suite of the product (fill reuse + ranked
# queue appends), A/B of the K-slider fill skip, PMC passes (refresh
# pmc_latest.json with the dual-issue counter), a default bench run.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_e.log; }
V=distributed-chess_amd/build/var
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_e.log 2>&1 || { tail -30 $O/pytest_gpu_e.log; exit 1; }
tail -2 $O/pytest_gpu_e.log
step ab-ref7
LEGS=ref7 timeout -k 10 400 python -u tools/ab_perft_time.py 6 $V/r4_prod/libdchess.so $V/r4_ks_reuse/libdchess.so > $O/ab_ref7_e.jsonl 2>&1 || { tail $O/ab_ref7_e.jsonl; exit 2; }
tail -1 $O/ab_ref7_e.jsonl
step bench
timeout -k 10 400 python -u bench.py > $O/bench_e.json 2> $O/bench_e.err || { tail -20 $O/bench_e.err; exit 3; }
step pmc
STAGES=pmc bash tools/gpu_round.sh || exit 4
step done
