#!/bin/bash
# Round-4 session Q: where the live validator's call time goes (mailbox probe
# poll shapes A/C/D/E, twice each), then the C-ABI probe of the product.
O=gpurun_out/r4
for r in 1 2; do
  for m in A C D E; do
    timeout -k 10 30 ./tools/live_mem_probe $m 5000 >> $O/live_mem_probe_q.jsonl 2>&1 || { echo "probe $m rc=$?" >> $O/live_mem_probe_q.jsonl; exit 2; }
  done
done
timeout -k 10 60 ./tools/latency_probe 5000 >> $O/live_mem_probe_q.jsonl 2>&1 || exit 3
cat $O/live_mem_probe_q.jsonl
