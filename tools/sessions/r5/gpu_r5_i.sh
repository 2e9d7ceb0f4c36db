#!/bin/bash
# Round-5 session I: the FIDE leaf count alone (minimal
# victim, reproducer revision's headers) beside co-resident noise waves.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
M=/tmp/dchess_map_$$
mkdir -p $O $M
DCHESS_LIB=$V/t_king_r4_diag1/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py --save-map $M kiwipete pos6 \
  >> $O/count_victim_i.jsonl 2>> $O/count_victim_i.err || exit 1
timeout -k 10 600 python -u tools/diag/count_victim.py --map $M --libs r4tab --kinds=-1,1,12,0 >> $O/count_victim_i.jsonl 2>> $O/count_victim_i.err || exit 1
rm -rf $M
cut -c1-400 $O/count_victim_i.jsonl
