#!/bin/bash
# Round-5 session T: the batch perft (dc_perft_batch: the FIDE suite as one tree)
# -- its GPU tests, the FIDE / REF perft tests around it, and the bench's FIDE legs.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_fide.py tests/test_gpu_ref.py > $O/pytest_t.log 2>&1 || { tail -40 $O/pytest_t.log; exit 1; }
tail -3 $O/pytest_t.log
timeout -k 10 300 python -u bench.py --only fidesuite,fide7,perft,perft6 --no-cpu > $O/bench_t.json 2> $O/bench_t.err || { tail -20 $O/bench_t.err; exit 2; }
python3 -c "
import json; d=json.load(open('$O/bench_t.json'))
print('perft7', d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'perft6', d['perft6']['ms_per_step'])
for k in ('fide_perft7','fide_suite_d5'):
    x=d.get(k); print(k, x.get('ms_per_step'), x.get('sequential_ms_per_step'), x.get('final_kernel_ms'), (x.get('roofline') or {}).get('frac'), x.get('batch','')[:40])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_t -o t --output-format csv -- python3 bench.py --only fidesuite --no-cpu --profile-only > $O/prof_t.log 2>&1 || { tail -20 $O/prof_t.log; exit 3; }
head -8 $O/prof_t/t_kernel_stats.csv | cut -c1-160
