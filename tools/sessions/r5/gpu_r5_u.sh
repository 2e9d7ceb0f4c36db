#!/bin/bash
# Round-5 session U: perft steps split over concurrent contexts (tools/overlap_perft.py).
O=gpurun_out/r5
mkdir -p $O
for c in 2 3; do
  timeout -k 10 120 python -u tools/overlap_perft.py --ctx $c --depth 7 --steps 48 >> $O/overlap_u.jsonl 2>> $O/overlap_u.err || { tail $O/overlap_u.err; exit 1; }
  timeout -k 10 120 python -u tools/overlap_perft.py --ctx $c --depth 6 --steps 96 >> $O/overlap_u.jsonl 2>> $O/overlap_u.err || { tail $O/overlap_u.err; exit 1; }
done
cat $O/overlap_u.jsonl
