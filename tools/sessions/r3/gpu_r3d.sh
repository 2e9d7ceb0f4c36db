#!/bin/bash
# Round-3 session d: the group-wise recount of the final stage (DC_C2C_DIAGQ=1,
# product) against the round-3 v2 final stage (build/var/lib_nodq.so): the
# perft GPU tests (goldens, divide, refcpu-pinned subtrees, K4 perft(8)/(9),
# odd positions), then the perft legs of both builds, alternating.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref.py tests/test_gpu_dfs.py -x -q --timeout 200 --timeout-method thread > $O/pytest_dq.log 2>&1 || { tail -30 $O/pytest_dq.log; exit 1; }
tail -2 $O/pytest_dq.log
NODQ=$PWD/distributed-chess_amd/build/var/lib_nodq.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_dq_$r.json 2>>$O/bench_dq.err || { tail $O/bench_dq.err; exit 2; }
  DCHESS_LIB=$NODQ timeout -k 10 200 python -u bench.py --only perft,perft6,perft8 --no-cpu --steps 20 > $O/bench_nodq_$r.json 2>>$O/bench_dq.err || exit 3
done
for f in $O/bench_dq_1.json $O/bench_nodq_1.json $O/bench_dq_2.json $O/bench_nodq_2.json; do
  python -c "import json,sys;d=json.load(open('$f'));print('$f', d['ms_per_step'], d.get('roofline',{}).get('kernel_avg_ms'), d.get('perft6',{}).get('ms_per_step'), d.get('perft8',{}).get('ms_per_step'))"
done
# replay: lazy-vacate mailbox (product) against the round-3 v2 replay (lib_r4nolazy)
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay_full.py tests/test_gpu_replay_info.py -x -q --timeout 200 --timeout-method thread > $O/pytest_lazy.log 2>&1 || { tail -30 $O/pytest_lazy.log; exit 4; }
tail -2 $O/pytest_lazy.log
NOLAZY=$PWD/distributed-chess_amd/build/var/lib_r4nolazy.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_lazy_$r.json 2>>$O/bench_dq.err || exit 5
  DCHESS_LIB=$NOLAZY timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_nolazy_$r.json 2>>$O/bench_dq.err || exit 6
done
for f in $O/bench_lazy_1.json $O/bench_nolazy_1.json $O/bench_lazy_2.json $O/bench_nolazy_2.json; do
  python -c "import json;d=json.load(open('$f'))['replay'];print('$f', d['kernel_avg_ms'], d['replay_parity'])"
done
