#!/bin/bash
# Round-3 generator check: its GPU tests (goldens incl. the 10M-game C4 moves
# SHA-256), then the replay leg (end-to-end with generation) of the product
# build, and the A/B build's round-2 generator (DC_GEN=2) for comparison.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_replay_full.py -x -q --timeout 200 --timeout-method thread > $O/pytest_gen.log 2>&1 || { tail -30 $O/pytest_gen.log; exit 1; }
tail -2 $O/pytest_gen.log
timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_gen_v3.json 2>$O/bench_gen.err || { cat $O/bench_gen.err; exit 2; }
DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so DC_GEN=2 timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_gen_v2.json 2>>$O/bench_gen.err || exit 3
for v in v3 v2; do python -c "import json;d=json.load(open('$O/bench_gen_$v.json'))['replay'];print('$v', d['end_to_end']['ms_per_step'], d['end_to_end']['gen_kernel_avg_ms'], d['kernel_avg_ms'], d['replay_parity'])"; done
