#!/bin/bash
# Round 4, session ZE: where the live validator's n = 1 time goes -- the
# product against a build whose validate answers without computing
# (DC_LIVE_EXP=1), alternated, tools/latency_probe at the C ABI.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
V=distributed-chess_amd/build/var/live1
LD_LIBRARY_PATH=$V ldd tools/latency_probe | grep dchess > $O/live_exp_ze.txt
for r in 1 2 3; do
  echo "product $(timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_exp_ze.txt || exit 1
  echo "nocompute $(LD_LIBRARY_PATH=$V timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_exp_ze.txt || exit 2
done
cat $O/live_exp_ze.txt
