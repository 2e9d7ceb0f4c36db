#!/bin/bash
# Round-3 GPU session: product tests, perft bench, the spill-free build's
# struct-of-arrays variant, the per-group logs of the failing round-2 layout,
# and the 48-byte-record layout's perft step.  Each step has its own limit.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u bench.py --only perft --no-cpu --steps 40 > $O/bench_perft_otid.json 2>$O/bench.err || { cat $O/bench.err; exit 2; }
cat $O/bench_perft_otid.json | python -c "import json,sys;d=json.load(sys.stdin);print('otid', d['ms_per_step'], d['kernels_ms_per_step'])"
DCHESS_LIB=$PWD/distributed-chess_amd/build/var/lib_rec.so timeout -k 10 120 python -u bench.py --only perft --no-cpu --steps 40 > $O/bench_perft_rec.json 2>>$O/bench.err || exit 3
cat $O/bench_perft_rec.json | python -c "import json,sys;d=json.load(sys.stdin);print('rec', d['ms_per_step'], d['kernels_ms_per_step'])"
TAG=soa_otid DCHESS_LIB=$PWD/distributed-chess_amd/build/var/lib_soa_otid.so timeout -k 10 120 python -u tools/c2c_diag.py 4 > $O/c2c_diag_soa_otid.jsonl 2>&1 || exit 4
cat $O/c2c_diag_soa_otid.jsonl | python -c "import json,sys;[print(d['tag'],d['depth'],d['run'],d['delta']) for d in map(json.loads,sys.stdin)]"
for v in soa_log aos_log; do TAG=$v DCHESS_LIB=$PWD/distributed-chess_amd/build/var/lib_$v.so timeout -k 10 120 python -u tools/c2c_groups.py 6 3 >> $O/c2c_groups.jsonl 2>&1 || exit 5; done
cat $O/c2c_groups.jsonl
