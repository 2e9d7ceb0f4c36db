#!/bin/bash
# Round 4, session ZD: FIDE depth 5 with the top kernel one ply short (the
# suite positions' ply 3 made on every CU): FIDE tests of the product, then a
# same-box A/B against the committed product (fide7 + suite legs).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fide.py -x -v --timeout 300 --timeout-method thread > $O/pytest_fide_zd.log 2>&1 || { tail -40 $O/pytest_fide_zd.log; exit 1; }
tail -2 $O/pytest_fide_zd.log
LEGS=fide7,suite timeout -k 10 500 python -u tools/ab_perft_time.py 3 distributed-chess_amd/build/var/head/libdchess.so distributed-chess_amd/libdchess.so > $O/ab_top_zd.jsonl 2>&1 || { tail $O/ab_top_zd.jsonl; exit 3; }
tail -1 $O/ab_top_zd.jsonl
