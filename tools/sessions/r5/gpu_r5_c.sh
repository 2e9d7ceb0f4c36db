#!/bin/bash
# Round-5 session C (diagnostics) on the round-4 reproducer
# (dc_perft + dc_api at bc27e78, -DDC_FIDE_TAB=1 -DDC_FIDE_TAB_PARTS=1):
#  1. the map of every final-stage child from the full-record build (exact);
#  2. the count-only build (one dword per child) read against the map, twice;
#  3. the failing build without inline-asm shifts;
#  4. the failing build under HIP CU masks (with the CU count HIP reports);
#  5. the failing build at depth 6 (final-stage chunks full).
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
M=/tmp/dchess_dmap_$$
mkdir -p $O $M
chk() { timeout -k 10 180 python tools/fide_check.py "$@" >> $O/fide_check_c.jsonl 2>> $O/fide_check_c.err; }
DCHESS_LIB=$V/t_king_r4_diag1/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py --save-map $M kiwipete pos5 pos6 \
  >> $O/child_diag_c.jsonl 2>> $O/child_diag_c.err || exit 1
for r in 1 2; do
  DCHESS_LIB=$V/t_king_r4_diagk/libdchess.so timeout -k 10 300 python -u tools/fide_child_diag.py --kmap $M kiwipete pos5 pos6 \
    >> $O/child_diag_c.jsonl 2>> $O/child_diag_c.err || exit 1
done
rm -rf $M
DCHESS_LIB=$V/t_king_r4/libdchess.so chk || exit 1
for r in 1 2; do DCHESS_LIB=$V/t_king_r4_pad3/libdchess.so chk || exit 1; done
for m in 0x1 0x3 0xf 0xff 0xffff 0x5555555555555555 0xaaaaaaaaaaaaaaaa; do
  ROC_GLOBAL_CU_MASK=$m timeout -k 10 60 python -c "import torch,json; print(json.dumps({'cu_mask': '$m', 'cus': torch.cuda.get_device_properties(0).multi_processor_count}))" >> $O/fide_check_c.jsonl 2>> $O/fide_check_c.err || exit 1
  ROC_GLOBAL_CU_MASK=$m DCHESS_LIB=$V/t_king_r4/libdchess.so chk kiwipete pos5 pos6 || exit 1
done
DCHESS_LIB=$V/t_king_r4/libdchess.so chk --depth 6 kiwipete pos4 pos6 || exit 1
cut -c1-2500 $O/child_diag_c.jsonl
cat $O/fide_check_c.jsonl
