#!/bin/bash
# Round-3 session l: the sliced perft(9) path without the in-kernel result copy
# sliced fused final stage and through K4, and both fallbacks; (2) the repeat
# path's result copy fused into k_count3c's last block against the HEAD
# build before it (build/var/lib_head.so), perft legs alternating; (3) the
# perft(9) leg (both paths).
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_dfs.py -x -v --timeout 300 --timeout-method thread > $O/pytest_l.log 2>&1 || { tail -30 $O/pytest_l.log; exit 1; }
tail -1 $O/pytest_l.log
HEADLIB=$PWD/distributed-chess_amd/build/var/lib_head.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_l_new_$r.json 2>>$O/bench_l.err || { tail $O/bench_l.err; exit 2; }
  DCHESS_LIB=$HEADLIB timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_l_head_$r.json 2>>$O/bench_l.err || exit 3
done
for f in $O/bench_l_*_?.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4), round(d['perft6']['ms_per_step'],4), round(d['perft8']['ms_per_step'],3))"
done
timeout -k 10 300 python -u bench.py --only perft9 --no-cpu > $O/bench_l9.json 2>>$O/bench_l.err || { tail $O/bench_l.err; exit 4; }
python -c "
import json;x=json.load(open('$O/bench_l9.json'))['perft9']
print('perft9', x['path'], round(x['ms_per_step'],2), '%.3e'%x['value'], x['parity'], 'k4', round(x['k4']['ms_per_step'],2), '%.3e'%x['k4']['value'])
"
