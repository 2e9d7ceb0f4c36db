#!/bin/bash
# Round-5 session W: perft(7) steps over 2 contexts with and without torch's
# runtime initialised first, and with more hardware queues per process.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/overlap_w.jsonl
for args in "--ctx 2 --steps 20" "--ctx 2 --steps 20 --torch" "--ctx 3 --steps 21 --torch"; do
  timeout -k 10 120 python -u tools/overlap_perft.py --depth 7 $args >> $O/overlap_w.jsonl 2>> $O/overlap_w.err || { tail $O/overlap_w.err; exit 1; }
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/overlap_perft.py --depth 7 $args >> $O/overlap_w.jsonl 2>> $O/overlap_w.err || { tail $O/overlap_w.err; exit 1; }
done
cat $O/overlap_w.jsonl
