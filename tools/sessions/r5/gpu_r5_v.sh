#!/bin/bash
# Round-5 session V: the bench with repeated perft steps split over concurrent
# contexts (bench.py perft_streams), default run and a 1-stream reference.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench_v.json 2> $O/bench_v.err || { tail -20 $O/bench_v.err; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu --only perft,perft6,fidesuite --perft-streams 1 > $O/bench_v1.json 2> $O/bench_v1.err || { tail -20 $O/bench_v1.err; exit 2; }
python3 -c "
import json
for f in ('$O/bench_v.json','$O/bench_v1.json'):
    d=json.load(open(f)); print(f, 'perft7', round(d['value']/1e12,3), d['ms_per_step'], d['config'].get('streams_per_gpu'), 'kernel', d['roofline']['kernel_avg_ms'], d['roofline']['frac'])
    print('  perft6', d['perft6']['ms_per_step'], 'suite', d.get('fide_suite_d5',{}).get('ms_per_step'), (d.get('fide_suite_d5',{}).get('roofline') or {}).get('frac'))"
