#!/bin/bash
# Round-3 session b: the bench's N-rank path rehearsed with 2 gloo ranks on one
# GPU (FIDE legs included), then the PMC passes (refreshed W for every leg).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
DC_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu --replay-steps 1 --hash-steps 1 --tx-steps 1 > $O/gloo2_r3.json 2> $O/gloo2_r3.err || { tail -30 $O/gloo2_r3.err; exit 1; }
python -c "import json;d=json.load(open('$O/gloo2_r3.json'));print('gloo2', d['value'], d['n_gpus'], d.get('fide_perft7',{}).get('parity'), d['replay']['replay_parity'])"
STAGES="pmc" bash tools/gpu_round.sh || exit 2
