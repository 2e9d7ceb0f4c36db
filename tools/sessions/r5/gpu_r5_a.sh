#!/bin/bash
# Round-5 session A (diagnostics): per-child records of the
# failing FIDE table build (-DDC_FIDE_TAB=1 -DDC_FIDE_TAB_PARTS=1) recounted
# by fastcpu, a product-build control, and the failing build without inline
# asm shifts / without the otid asm.
O=gpurun_out/r5
V=distributed-chess_amd/build/var
mkdir -p $O
for v in r5_prod_diag1 r5_diag1 r5_diag2; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py kiwipete pos5 pos6 \
    >> $O/child_diag_a.jsonl 2>> $O/child_diag_a.err || exit 1
done
for v in r5_wrong r5_wrong_pad3 r5_wrong_livetid r5_wrong r5_wrong_pad3 r5_wrong_livetid; do
  DCHESS_LIB=$PWD/$V/$v/libdchess.so timeout -k 10 120 python tools/fide_check.py >> $O/fide_check_a.jsonl 2>> $O/fide_check_a.err || exit 1
done
cut -c1-600 $O/child_diag_a.jsonl
cat $O/fide_check_a.jsonl
