#!/bin/bash
# Round 6, session 3: k_count3c 64-word tail groups A/B (DC_C3C_TAIL=1 in
# libdchess_c3tail.so against the product build): REF perft parity on the
# variant, then one-context / two-context perft(7), perft(6) and shard 0 of 8.
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
NEW=$PWD/distributed-chess_amd/libdchess.so EV=$PWD/distributed-chess_amd/libdchess_c3tail.so
DCHESS_LIB=$EV timeout -k 10 400 python -u -m pytest tests/test_gpu_ref.py -x -q --timeout 200 --timeout-method thread > $O/pytest_c3tail.log 2>&1 || { tail -30 $O/pytest_c3tail.log; exit 1; }
tail -2 $O/pytest_c3tail.log
for v in base even base even; do
  L=$NEW; [ $v = even ] && L=$EV
  for args in "--depth 7" "--depth 6 --steps 64" "--depth 7 --shards 8 --steps 64"; do
    DCHESS_LIB=$L timeout -k 10 120 python -u tools/overlap_perft.py --ctx 2 --reps 3 $args > $O/ov.json 2> $O/ov.err || { tail $O/ov.err; exit 2; }
    echo "$v $args $(tail -1 $O/ov.json)" | tee -a $O/ab_c3tail.jsonl | cut -c1-400
  done
done
echo done
