#!/bin/bash
# Round-5 session Z2: chunk size rule of the dynamic k_count2b on the FIDE
# suite batch (one context, alternating builds) and FIDE perft(7).
O=gpurun_out/r5
mkdir -p $O
rm -f $O/ab_z2.jsonl
for r in 1 2 3; do
  for lib in $PWD/distributed-chess_amd/build/abq/q0/libdchess.so $PWD/distributed-chess_amd/libdchess.so $PWD/distributed-chess_amd/build/abq/dyn0/libdchess.so; do
    DCHESS_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --only fidesuite,fide7 --perft-streams 1 > $O/b_z2.json 2>> $O/b_z2.err || { tail $O/b_z2.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_z2.json')); s=d['fide_suite_d5']; f=d['fide_perft7']
print(json.dumps({'lib': '$lib'.split('/')[-2], 'round': $r, 'suite_ms': s['ms_per_step'], 'suite_final_ms': s['final_kernel_ms'], 'seq_ms': s.get('sequential_ms_per_step'), 'fide7_ms': f['ms_per_step']}))" >> $O/ab_z2.jsonl
  done
done
cat $O/ab_z2.jsonl
