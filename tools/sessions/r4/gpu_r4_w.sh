#!/bin/bash
# Round-4 session W (diagnostics): the kAtt king set in the FIDE analysis
# (wrong, run-to-run different counts on many CUs) with (a) the load waited
# for at once, (b) the table address in VGPRs; the broken build once more.
O=gpurun_out/r4
V=distributed-chess_amd/build/var
mkdir -p $O
for v in t_king_wait t_king_wait t_king_vaddr t_king_vaddr t_king; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 120 python tools/fide_check.py >> $O/fide_diag_w.jsonl 2>&1 || exit 1
done
cat $O/fide_diag_w.jsonl
