#!/bin/bash
# Round-3 session f: product (group-wise recount queue, tag and orthogonal
# mask read with the candidate's record) against the round-3 v2 final stage
# (lib_nodq), perft legs alternating; then the stall-reason PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref.py -k perft -x -q --timeout 200 --timeout-method thread > $O/pytest_f.log 2>&1 || { tail -30 $O/pytest_f.log; exit 1; }
tail -1 $O/pytest_f.log
NODQ=$PWD/distributed-chess_amd/build/var/lib_nodq.so
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_f_dq_$r.json 2>>$O/bench_f.err || { tail $O/bench_f.err; exit 2; }
  DCHESS_LIB=$NODQ timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_f_nodq_$r.json 2>>$O/bench_f.err || exit 3
done
for f in $O/bench_f_*_?.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4), round(d['perft6']['ms_per_step'],4), round(d['perft8']['ms_per_step'],3))"
done
STALL_ARGS="--steps 3 --warmup 1 --no-cpu --profile-only --only perft" bash tools/pmc_stall.sh > $O/stallsum_f.txt 2>&1 || { tail $O/stallsum_f.txt; exit 4; }
cat $O/stallsum_f.txt
