#!/bin/bash
# Round-5 session X: concurrent contexts at perft(8) and for the FIDE legs' depth.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/overlap_x.jsonl
timeout -k 10 200 python -u tools/overlap_perft.py --depth 8 --ctx 2 --steps 6 --reps 2 >> $O/overlap_x.jsonl 2>> $O/overlap_x.err || { tail $O/overlap_x.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --only fide7 --perft-streams 3 > $O/bench_x3.json 2> $O/bench_x3.err || { tail $O/bench_x3.err; exit 2; }
python3 -c "
import json; d=json.load(open('$O/bench_x3.json')); print('fide7 3 streams', d['fide_perft7']['ms_per_step'])"
cat $O/overlap_x.jsonl
