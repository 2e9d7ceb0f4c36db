#!/bin/bash
# Round-5 session AB: one rank's work at N = 4 and 8 (shard 0 of N) over 1-4 contexts.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/overlap_ab.jsonl
for sh in 4 8; do
  for c in 2 3 4; do
    timeout -k 10 120 python -u tools/overlap_perft.py --depth 7 --shards $sh --ctx $c --steps 48 --reps 2 >> $O/overlap_ab.jsonl 2>> $O/overlap_ab.err || { tail $O/overlap_ab.err; exit 1; }
  done
done
cat $O/overlap_ab.jsonl
