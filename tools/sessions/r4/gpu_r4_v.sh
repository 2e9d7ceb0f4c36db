#!/bin/bash
# Round-4 session V (diagnostics): the kAtt king set in the FIDE analysis with
# the sniper gate off (no __ballot in analyse), twice on the full GPU.
O=gpurun_out/r4
V=distributed-chess_amd/build/var
mkdir -p $O
for r in 1 2; do DCHESS_LIB=$PWD/$V/t_king_nosnip/libdchess.so timeout -k 10 120 python tools/fide_check.py >> $O/fide_diag_v.jsonl 2>&1 || exit 1; done
cat $O/fide_diag_v.jsonl
