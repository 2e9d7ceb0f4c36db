#!/bin/bash
# Round 4, session Z: the FIDE final stage's simple-child split (k_count2b
# kSplit): FIDE parity tests (published tables, deep), then a same-box A/B of
# the split against the pre-split build (fide7 + suite legs, parity checked
# on every step).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fide.py -x -v --timeout 300 --timeout-method thread > $O/pytest_fide_z.log 2>&1 || { tail -40 $O/pytest_fide_z.log; exit 1; }
tail -3 $O/pytest_fide_z.log
LEGS=fide7,suite timeout -k 10 500 python -u tools/ab_perft_time.py 3 distributed-chess_amd/build/var/r4base/libdchess.so distributed-chess_amd/libdchess.so > $O/ab_split_z.jsonl 2>&1 || { tail $O/ab_split_z.jsonl; exit 3; }
tail -1 $O/ab_split_z.jsonl
