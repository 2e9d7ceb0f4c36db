#!/bin/bash
# Round-4 session R: where the live validator's call time goes (mailbox probe
# poll shapes A/C/D/E, twice each) and the C-ABI probe of the product; then
# parity + same-box A/B of the sniper-gated FIDE pin scans (FIDE legs).
O=gpurun_out/r4
V=distributed-chess_amd/build/var
mkdir -p $O
for r in 1 2; do
  for m in A C D E; do
    timeout -k 10 30 ./tools/live_mem_probe $m 5000 >> $O/live_mem_probe_r.jsonl 2>&1 || { echo "probe $m rc=$?" >> $O/live_mem_probe_r.jsonl; exit 2; }
  done
done
timeout -k 10 60 ./tools/latency_probe 5000 >> $O/live_mem_probe_r.jsonl 2>&1 || exit 3
cat $O/live_mem_probe_r.jsonl
TAG=r LIB_A=$V/r4_nosniper/libdchess.so LIB_B=$V/r4_sniper/libdchess.so LEGS=fide7,suite ROUNDS=4 SKIP=prof,bench bash tools/gpu_ab_session.sh
