#!/bin/bash
# Round-4 session P: parity + same-box A/B of the 8-run batch graph, the bench,
# k_expand_top's per-ply timeline (A/B build), and the mailbox ping-pong probe
# (request word in pinned host memory vs fine-grained device memory).
V=distributed-chess_amd/build/var
O=gpurun_out/r4
TAG=p LIB_A=$V/r4_nobatch/libdchess.so LIB_B=$V/r4_batch/libdchess.so ROUNDS=6 SKIP=prof bash tools/gpu_ab_session.sh || exit $?
DEPTH=7 DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so timeout -k 10 120 python tools/top_trace.py > $O/top_trace_p.json 2>&1 || { cat $O/top_trace_p.json; exit 8; }
cat $O/top_trace_p.json
for m in A B A B; do
  timeout -k 10 30 ./tools/live_mem_probe $m 5000 >> $O/live_mem_probe_p.jsonl 2>&1 || { echo "probe $m rc=$?" >> $O/live_mem_probe_p.jsonl; break; }
done
cat $O/live_mem_probe_p.jsonl
