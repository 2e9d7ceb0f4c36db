#!/bin/bash
# Round-5 session AN: W rays on the 180-degree rotated board (DC_GEN_WROT) in the generator counts.
# Generator / replay parity first (C4 moves SHA-256 and the replay goldens),
# then the bench's replay leg (end to end with generation) alternating builds.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/ab_an.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ref.py tests/test_gpu_replay_full.py tests/test_gpu_replay_info.py tests/test_statehash.py -k "gen or replay or hash or sha" > $O/t_an.log 2>&1 || { tail -30 $O/t_an.log; exit 1; }
tail -2 $O/t_an.log
for r in 1 2 3; do
  for lib in $PWD/distributed-chess_amd/build/abq/gen_old/libdchess.so $PWD/distributed-chess_amd/libdchess.so; do
    DCHESS_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --only replay > $O/b_an.json 2>> $O/b_an.err || { tail $O/b_an.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_an.json'))['replay']; e=d['end_to_end']
print(json.dumps({'lib': '$lib'.split('/')[-2], 'round': $r, 'gen_kernel_ms': e['gen_kernel_avg_ms'], 'e2e_ms': e['ms_per_step'], 'parity': d['replay_parity'], 'digest_xor': d['combined_stats']['digest_xor']}))" >> $O/ab_an.jsonl
  done
done
cat $O/ab_an.jsonl
