#!/bin/bash
# Round-4 session U (diagnostics): the FIDE final stage with the king attack
# set from kAtt gives wrong, run-to-run different suite counts.  Repeat it,
# run it on one CU, and with the table load issued outside the branch.
O=gpurun_out/r4
V=distributed-chess_amd/build/var
mkdir -p $O
run() { timeout -k 10 120 python tools/fide_check.py >> $O/fide_diag_u.jsonl 2>&1 || { echo "rc=$? $*" >> $O/fide_diag_u.jsonl; exit 1; }; }
for r in 1 2 3; do DCHESS_LIB=$PWD/$V/t_king/libdchess.so run; done
ROC_GLOBAL_CU_MASK=0x1 DCHESS_LIB=$PWD/$V/t_king/libdchess.so run
ROC_GLOBAL_CU_MASK=0xffffffff DCHESS_LIB=$PWD/$V/t_king/libdchess.so run
for r in 1 2; do DCHESS_LIB=$PWD/$V/t_king_unc/libdchess.so run; done
DCHESS_LIB=$PWD/$V/r4_fidenotab/libdchess.so run
cat $O/fide_diag_u.jsonl
