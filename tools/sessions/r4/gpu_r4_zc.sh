#!/bin/bash
# Round 4, session ZC: FIDE split with the semi-simple class (enumerated
# counting pass, DC_FIDE_SPLIT=1) against the committed product (set-wise
# counting pass, no semi class); FIDE tests of the variant first.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
DCHESS_LIB=$PWD/distributed-chess_amd/build/var/semi1/libdchess.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fide.py -x -v --timeout 300 --timeout-method thread > $O/pytest_fide_zc.log 2>&1 || { tail -40 $O/pytest_fide_zc.log; exit 1; }
tail -2 $O/pytest_fide_zc.log
LEGS=fide7,suite timeout -k 10 500 python -u tools/ab_perft_time.py 3 distributed-chess_amd/build/var/head/libdchess.so distributed-chess_amd/build/var/semi1/libdchess.so > $O/ab_semi_zc.jsonl 2>&1 || { tail $O/ab_semi_zc.jsonl; exit 3; }
tail -1 $O/ab_semi_zc.jsonl
