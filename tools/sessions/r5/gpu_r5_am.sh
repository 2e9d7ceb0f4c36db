#!/bin/bash
# Round-5 session AM: state hash with the replay kernel's per-ply info pass first (DC_HASH_PRE) against the single kernel.
# State-hash parity first, then the bench's hash leg alternating builds.
O=gpurun_out/r5
mkdir -p $O
rm -f $O/ab_am.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_statehash.py tests/test_gpu_replicas.py tests/test_gpu_replay_info.py > $O/t_am.log 2>&1 || { tail -30 $O/t_am.log; exit 1; }
tail -2 $O/t_am.log
# every hash of 200k bench games, both builds
for lib in $PWD/distributed-chess_amd/build/abq/hash_nopre/libdchess.so $PWD/distributed-chess_amd/libdchess.so; do
  DCHESS_LIB=$lib timeout -k 10 120 python3 - $O/h_$(basename $(dirname $lib)).npy <<'PY' || exit 1
import sys, numpy as np
sys.path.insert(0, "distributed-chess_amd")
import dchess
e = dchess.Engine(0)
n, P = 200000, 80
mv = e.gen_games(0x5EED20241022, 0, n, P, 32)
names = [(f"white{g}", "bl\"ack" + str(g)) for g in range(n)]
np.save(sys.argv[1], e.state_hash(mv, names))
PY
done
python3 -c "
import numpy as np; a=np.load('$O/h_hash_nopre.npy'); b=np.load('$O/h_distributed-chess_amd.npy'); assert a.shape==b.shape and (a==b).all(); print('200k hashes identical across builds')" || exit 1
for r in 1 2 3; do
  for lib in $PWD/distributed-chess_amd/build/abq/hash_nopre/libdchess.so $PWD/distributed-chess_amd/libdchess.so; do
    DCHESS_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --only hash > $O/b_am.json 2>> $O/b_am.err || { tail $O/b_am.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_am.json'))['state_hash']
print(json.dumps({'lib': '$lib'.split('/')[-2], 'round': $r, 'ms': d['ms_per_step'], 'kernel_ms': d['kernel_avg_ms'], 'pre_ms': d.get('replay_prepass_ms'), 'value': d['value'], 'h0': d['first_hash'][:18]}))" >> $O/ab_am.jsonl
  done
done
cat $O/ab_am.jsonl
