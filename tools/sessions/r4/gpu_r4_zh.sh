#!/bin/bash
# Round 4, session ZH: fide_count computes the attack map only in waves with a
# king move or an open castling path (DC_FIDE_LAZY_DANGER=1; =2 also in the
# split's count and enumeration passes): the FIDE GPU tests on both builds,
# then a same-box A/B against the product (=0).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
for v in lazy1 lazy2; do
  DCHESS_LIB=$PWD/distributed-chess_amd/build/var/$v/libdchess.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fide.py -x -v --timeout 300 --timeout-method thread > $O/pytest_fide_zh_$v.log 2>&1 || { tail -30 $O/pytest_fide_zh_$v.log; exit 1; }
  tail -1 $O/pytest_fide_zh_$v.log
done
LEGS=fide7,suite timeout -k 10 600 python -u tools/ab_perft_time.py 3 distributed-chess_amd/libdchess.so distributed-chess_amd/build/var/lazy1/libdchess.so distributed-chess_amd/build/var/lazy2/libdchess.so > $O/ab_lazy_zh.jsonl 2>&1 || { tail $O/ab_lazy_zh.jsonl; exit 3; }
tail -1 $O/ab_lazy_zh.jsonl
