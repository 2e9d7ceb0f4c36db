#!/bin/bash
# Round-3 session j: the repeat path's result copy fused into k_count3c's last
# block (no k_copy_result launch), against the committed HEAD build
# (build/var/lib_head.so), perft legs alternating.
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_dfs.py -x -q --timeout 200 --timeout-method thread > $O/pytest_j.log 2>&1 || { tail -30 $O/pytest_j.log; exit 1; }
tail -1 $O/pytest_j.log
HEADLIB=$PWD/distributed-chess_amd/build/var/lib_head.so
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_j_new_$r.json 2>>$O/bench_j.err || { tail $O/bench_j.err; exit 2; }
  DCHESS_LIB=$HEADLIB timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_j_head_$r.json 2>>$O/bench_j.err || exit 3
done
for f in $O/bench_j_*_?.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4), round(d['perft6']['ms_per_step'],4), round(d['perft8']['ms_per_step'],3))"
done
