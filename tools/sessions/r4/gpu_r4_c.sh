#!/bin/bash
# Round-4 session C: full GPU parity suite of the current product, then same-box
# A/B timings (tools/ab_perft_time.py) of the round-4 kernel variants.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_c.log; }
V=distributed-chess_amd/build/var
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_c.log 2>&1 || { tail -30 $O/pytest_gpu_c.log; exit 1; }
tail -2 $O/pytest_gpu_c.log
step ab-ref7
LEGS=ref7 timeout -k 10 400 python -u tools/ab_perft_time.py 5 $V/r4_asm/libdchess.so $V/r4_sgpr/libdchess.so $V/r4_w5/libdchess.so > $O/ab_ref7.jsonl 2>&1 || { tail $O/ab_ref7.jsonl; exit 2; }
tail -1 $O/ab_ref7.jsonl
step ab-fide
LEGS=fide7,suite timeout -k 10 400 python -u tools/ab_perft_time.py 3 $V/r4_fide4/libdchess.so $V/r4_sgpr/libdchess.so > $O/ab_fide.jsonl 2>&1 || { tail $O/ab_fide.jsonl; exit 3; }
tail -1 $O/ab_fide.jsonl
step done
