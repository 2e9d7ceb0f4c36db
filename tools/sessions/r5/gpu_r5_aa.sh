#!/bin/bash
# Round-5 session AA: how many contexts per GPU for perft(6) / perft(7).
O=gpurun_out/r5
mkdir -p $O
rm -f $O/streams_aa.jsonl
for n in 2 3 4; do
  timeout -k 10 200 python -u bench.py --no-cpu --only perft,perft6 --perft-streams $n > $O/b_aa.json 2>> $O/b_aa.err || { tail $O/b_aa.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_aa.json')); print(json.dumps({'streams': $n, 'perft7_ms': d['ms_per_step'], 'perft6_ms': d['perft6']['ms_per_step']}))" >> $O/streams_aa.jsonl
done
cat $O/streams_aa.jsonl
