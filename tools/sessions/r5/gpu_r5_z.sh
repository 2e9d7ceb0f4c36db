#!/bin/bash
# Round-5 session Z: k_count2b with dynamic chunk scheduling (DC_C2B_DYN):
# FIDE parity, then a same-box A/B of the FIDE legs against the static split.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fide.py tests/test_gpu_batch.py tests/test_gpu_fide_split.py > $O/pytest_z.log 2>&1 || { tail -40 $O/pytest_z.log; exit 1; }
tail -2 $O/pytest_z.log
LEGS=fide7,suite timeout -k 10 500 python -u tools/ab_perft_time.py 3 $PWD/distributed-chess_amd/build/abq/dyn0/libdchess.so $PWD/distributed-chess_amd/libdchess.so > $O/ab_dyn_z.jsonl 2>&1 || { tail $O/ab_dyn_z.jsonl; exit 2; }
tail -1 $O/ab_dyn_z.jsonl
timeout -k 10 300 python -u bench.py --no-cpu --only fide7,fidesuite > $O/bench_z.json 2> $O/bench_z.err || { tail -20 $O/bench_z.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/bench_z.json'))
for k in ('fide_perft7','fide_suite_d5'):
    x=d[k]; print(k, x['ms_per_step'], x.get('final_kernel_ms'), (x.get('roofline') or {}).get('frac'))"
