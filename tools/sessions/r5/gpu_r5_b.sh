#!/bin/bash
# Round-5 session B (diagnostics): the round-4 reproducer
# rebuilt from its own revision (dc_perft + dc_api at bc27e78, -DDC_FIDE_TAB=1
# -DDC_FIDE_TAB_PARTS=1), plain and with the per-child records; the current
# source's table variant without the final-stage split.
O=gpurun_out/r5
V=distributed-chess_amd/build/var
mkdir -p $O
for v in t_king_r4 t_king_r4 r5_wrong_nosplit r5_wrong_nosplit; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 120 python tools/fide_check.py >> $O/fide_check_b.jsonl 2>> $O/fide_check_b.err || exit 1
done
for v in t_king_r4_diag1 t_king_r4_diag2; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py kiwipete pos5 pos6 \
    >> $O/child_diag_b.jsonl 2>> $O/child_diag_b.err || exit 1
done
cat $O/fide_check_b.jsonl
cut -c1-1500 $O/child_diag_b.jsonl
