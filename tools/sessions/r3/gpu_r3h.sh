#!/bin/bash
# Round-3 session h: REF perft(8) through the fused final stage with 64-bit
# move words (and K4 forced, DCHESS_PERFT_K4=1), the DFS tests, then the
# perft8 / perft9 bench legs.
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dfs.py -x -v --timeout 200 --timeout-method thread > $O/pytest_h.log 2>&1 || { tail -30 $O/pytest_h.log; exit 1; }
tail -3 $O/pytest_h.log
timeout -k 10 300 python -u bench.py --only perft,perft8,perft9 --no-cpu --steps 20 > $O/bench_h.json 2>$O/bench_h.err || { tail $O/bench_h.err; exit 2; }
python -c "
import json;d=json.load(open('$O/bench_h.json'))
print('d7', round(d['ms_per_step'],4))
for k in ('perft8','perft9'):
    x=d[k]; print(k, x.get('path'), round(x['ms_per_step'],3), '%.3e'%x['value'], x['parity'], x.get('dfs_kernel_ms'), (x.get('roofline') or {}).get('kernel_avg_ms'))
"
