#!/bin/bash
# Round-5 session Y: the quiet-children queue (DC_C2C_QQ): REF parity, then a
# same-box A/B of perft(7) against the build without it.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref.py tests/test_gpu_dfs.py tests/test_gpu_stress.py > $O/pytest_y.log 2>&1 || { tail -40 $O/pytest_y.log; exit 1; }
tail -2 $O/pytest_y.log
LEGS=ref7 timeout -k 10 400 python -u tools/ab_perft_time.py 5 $PWD/distributed-chess_amd/build/abq/qq0/libdchess.so $PWD/distributed-chess_amd/libdchess.so > $O/ab_qq_y.jsonl 2>&1 || { tail $O/ab_qq_y.jsonl; exit 2; }
tail -3 $O/ab_qq_y.jsonl
