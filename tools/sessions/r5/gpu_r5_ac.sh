#!/bin/bash
# Round-5 session AC: strided shards made from the top kernel's words (no
# one-workgroup board ply, no gather): sharded parity, then one rank's step.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref.py tests/test_gpu_fide.py tests/test_gpu_dfs.py tests/test_gpu_batch.py > $O/pytest_ac.log 2>&1 || { tail -40 $O/pytest_ac.log; exit 1; }
tail -2 $O/pytest_ac.log
rm -f $O/overlap_ac.jsonl
for sh in 4 8; do
  for c in 1 3; do
    timeout -k 10 120 python -u tools/overlap_perft.py --depth 7 --shards $sh --ctx $c --steps 48 --reps 2 >> $O/overlap_ac.jsonl 2>> $O/overlap_ac.err || { tail $O/overlap_ac.err; exit 2; }
  done
done
cat $O/overlap_ac.jsonl
