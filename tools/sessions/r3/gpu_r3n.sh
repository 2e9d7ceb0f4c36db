#!/bin/bash
# Round-3 session n: the round-2 failing build (tools/gpu_r3m.sh's tree) on
# perft(6)/(7) after 1.e4: which of side-to-move template and grid length
# goes with the error (tools/c2c_diag_e4.py).  All CUs, then one CU.
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
cd distributed-chess_amd/build/var/r2tree || exit 1
for cfg in BASE=1 ROC_GLOBAL_CU_MASK=0x1; do
  env $cfg TAG="$cfg" timeout -k 10 200 python -u tools/c2c_diag_e4.py 3 > $O/r2e4_${cfg//[=x]/_}.jsonl 2>$O/r2e4.err || { tail $O/r2e4.err; exit 2; }
  python -c "
import json
rs=[json.loads(l) for l in open('$O/r2e4_${cfg//[=x]/_}.jsonl')]
print('$cfg', [(r['depth'], r['delta']) for r in rs])
"
done
