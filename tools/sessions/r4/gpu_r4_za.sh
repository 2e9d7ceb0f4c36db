#!/bin/bash
# Round 4, session ZA: FIDE split, enumerated counting pass (product) against
# the set-wise counting pass (DC_FIDE_SPLIT=2), same box, parity every step.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
LEGS=fide7,suite timeout -k 10 500 python -u tools/ab_perft_time.py 3 distributed-chess_amd/libdchess.so distributed-chess_amd/build/var/split2/libdchess.so > $O/ab_split2_za.jsonl 2>&1 || { tail $O/ab_split2_za.jsonl; exit 3; }
tail -1 $O/ab_split2_za.jsonl
