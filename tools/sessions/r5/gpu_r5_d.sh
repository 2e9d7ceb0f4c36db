#!/bin/bash
# Round-5 session D (diagnostics) on the round-4 reproducer
# (dc_perft + dc_api at bc27e78, -DDC_FIDE_TAB=1 -DDC_FIDE_TAB_PARTS=1):
#  1. where blocks land under CU masks (tools/diag/cu_probe);
#  2. the failing build under masks that separate CU count from XCD count;
#  3. the same kernel (ISA identical) on chosen grids without a mask;
#  4. per-root-move errors and run-to-run spread in one process.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
chk() { timeout -k 10 180 python tools/fide_check.py "$@" >> $O/fide_check_d.jsonl 2>> $O/fide_check_d.err; }
for m in 0x3 0xf 0x101 0x11 0x1111 0x01010101 0x0f0f 0xff; do
  echo "{\"probe_mask\": \"$m\"}" >> $O/cu_probe_d.jsonl
  ROC_GLOBAL_CU_MASK=$m timeout -k 10 60 tools/diag/cu_probe >> $O/cu_probe_d.jsonl 2>&1 || exit 1
done
timeout -k 10 60 tools/diag/cu_probe 24 >> $O/cu_probe_d.jsonl 2>&1 || exit 1
for m in 0x101 0x01010101 0x11 0x1111 0x0f0f; do
  ROC_GLOBAL_CU_MASK=$m DCHESS_LIB=$V/t_king_r4/libdchess.so chk kiwipete pos5 pos6 || exit 1
done
for g in 3 6 12 24 48 96 384; do
  DC_DIAG_GRID=$g DCHESS_LIB=$V/t_king_r4_grid/libdchess.so chk kiwipete pos5 pos6 || exit 1
done
DCHESS_LIB=$V/t_king_r4/libdchess.so chk --divide --repeat 4 kiwipete pos6 || exit 1
cat $O/cu_probe_d.jsonl | cut -c1-400
cat $O/fide_check_d.jsonl | cut -c1-1500
