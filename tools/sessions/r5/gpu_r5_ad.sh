#!/bin/bash
# Round-5 session AD: FIDE slider fills cut to two per direction when no wave
# lane has an unpinned slider on a split source square (DC_FIDE_FILL2).
# FIDE parity first, then the bench's FIDE legs alternating builds.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/ab_ad.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fide_split.py tests/test_gpu_batch.py tests/test_gpu_fide.py > $O/t_ad.log 2>&1 || { tail -30 $O/t_ad.log; exit 1; }
tail -2 $O/t_ad.log
for r in 1 2 3; do
  for lib in $PWD/distributed-chess_amd/build/abq/fill2_off/libdchess.so $PWD/distributed-chess_amd/libdchess.so; do
    DCHESS_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --only fidesuite,fide7 > $O/b_ad.json 2>> $O/b_ad.err || { tail $O/b_ad.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_ad.json')); s=d['fide_suite_d5']; f=d['fide_perft7']
print(json.dumps({'lib': '$lib'.split('/')[-2], 'round': $r, 'suite_ms': s['ms_per_step'], 'suite_final_ms': s['final_kernel_ms'], 'fide7_ms': f['ms_per_step'], 'fide7_final_ms': f.get('final_kernel_ms')}))" >> $O/ab_ad.jsonl
  done
done
cat $O/ab_ad.jsonl
