#!/bin/bash
# Round-3 session m: the round-2 failing final stage (the whole round-2 tree,
# commit 3d8df08, built with -DDC_C2C_SOA=1: k_count3c spills 48 B/lane) under
# the ROCr scratch-management switches (tree: tools/build_r2tree.sh).  If a switch that changes how the
# runtime grows, limits or reclaims scratch makes perft(6) exact, the fault
# lies in scratch management, not in the kernel's code.  3 runs per setting.
# CFGS="ROC_GLOBAL_CU_MASK=0x1 ..." runs the same under a CU mask (fewer CUs,
# less concurrency) instead.
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
cd distributed-chess_amd/build/var/r2tree || exit 1
CFGS=${CFGS:-"BASE=1 HSA_NO_SCRATCH_RECLAIM=1 HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0 HSA_NO_SCRATCH_THREAD_LIMITER=1 HSA_SCRATCH_SINGLE_LIMIT=4294967296"}
for cfg in $CFGS; do
  env $cfg TAG="$cfg" timeout -k 10 120 python -u tools/c2c_diag.py 3 > $O/r2scratch_${cfg//[=x]/_}.jsonl 2>$O/r2scratch.err || { tail $O/r2scratch.err; exit 2; }
  python -c "
import json
rs=[json.loads(l) for l in open('$O/r2scratch_${cfg//[=x]/_}.jsonl')]
print('$cfg', [(r['depth'], r['delta']) for r in rs])
"
done
