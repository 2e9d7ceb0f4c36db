#!/bin/bash
# Round-3 session e: where k_count2c's time goes (A/B build, DC_FUSED3=0 so
# the final stage is k_count2c over ply-5 boards; DC_C2C_PHASE: 0 full,
# 5 no full/group recounts, 6 also no quiet-child pawn counts, 1 no children,
# 2 no enumeration either -- wrong counts except 0, timing only), then the
# stall-reason PMC passes of the product's perft step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
export DC_FUSED3=0
AB_VARIANTS="DC_C2C_PHASE=0 DC_C2C_PHASE=5 DC_C2C_PHASE=6 DC_C2C_PHASE=1 DC_C2C_PHASE=2 DC_C2C_PHASE=0" bash tools/ab_phase.sh || exit 1
unset DC_FUSED3
STALL_ARGS="--steps 3 --warmup 1 --no-cpu --profile-only --only perft" bash tools/pmc_stall.sh > $O/stall_summary.txt 2>&1 || { tail $O/stall_summary.txt; exit 2; }
cat $O/stall_summary.txt
