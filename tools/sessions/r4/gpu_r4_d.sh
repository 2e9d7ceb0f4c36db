#!/bin/bash
# Round-4 session D: A/B of the fill-reuse final stage, FIDE budgets, and the
# select micro-benchmark modes.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps_d.log; }
V=distributed-chess_amd/build/var
step ubench
timeout -k 10 120 ./tools/ubench/dual_issue > $O/ubench_dual_issue_v2.txt 2>&1 || { tail $O/ubench_dual_issue_v2.txt; exit 1; }
step ubench-pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/ubench_pmc_v2 -o p -- ./tools/ubench/dual_issue > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 2; }
step ab-ref7
LEGS=ref7 timeout -k 10 500 python -u tools/ab_perft_time.py 6 $V/r4_base/libdchess.so $V/r4_reuse/libdchess.so $V/r4_rank/libdchess.so $V/r4_rank_reuse/libdchess.so > $O/ab_ref7_d.jsonl 2>&1 || { tail $O/ab_ref7_d.jsonl; exit 3; }
tail -1 $O/ab_ref7_d.jsonl
step ab-fide
LEGS=fide7,suite timeout -k 10 400 python -u tools/ab_perft_time.py 3 $V/r4_fide4/libdchess.so $V/r4_base/libdchess.so > $O/ab_fide_d.jsonl 2>&1 || { tail $O/ab_fide_d.jsonl; exit 4; }
tail -1 $O/ab_fide_d.jsonl
step done
