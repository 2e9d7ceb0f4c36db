#!/bin/bash
# Round-5 session AL: k_count2b chunks of equal size <= 256 (DC_C2B_BAL) on the FIDE suite batch and FIDE perft(7).
# FIDE parity first, then the bench's FIDE legs alternating builds.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/ab_al.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fide_split.py tests/test_gpu_batch.py tests/test_gpu_fide.py > $O/t_al.log 2>&1 || { tail -30 $O/t_al.log; exit 1; }
tail -2 $O/t_al.log
for r in 1 2 3; do
  for lib in $PWD/distributed-chess_amd/build/abq/bal/libdchess.so $PWD/distributed-chess_amd/libdchess.so; do
    DCHESS_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --only fidesuite,fide7 > $O/b_al.json 2>> $O/b_al.err || { tail $O/b_al.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_al.json')); s=d['fide_suite_d5']; f=d['fide_perft7']
print(json.dumps({'lib': '$lib'.split('/')[-2], 'round': $r, 'suite_ms': s['ms_per_step'], 'suite_final_ms': s['final_kernel_ms'], 'fide7_ms': f['ms_per_step'], 'fide7_final_ms': f.get('final_kernel_ms')}))" >> $O/ab_al.jsonl
  done
done
cat $O/ab_al.jsonl
