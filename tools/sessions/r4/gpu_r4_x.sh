#!/bin/bash
# Round-4 session X (diagnostics): the kAtt king set in the FIDE analysis with
# the sniper gate as per-lane branches instead of __ballot-uniform ones.
O=gpurun_out/r4
V=distributed-chess_amd/build/var
mkdir -p $O
for v in t_king_lanebr t_king_lanebr t_king_lanebr; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 120 python tools/fide_check.py >> $O/fide_diag_x.jsonl 2>&1 || exit 1
done
cat $O/fide_diag_x.jsonl
