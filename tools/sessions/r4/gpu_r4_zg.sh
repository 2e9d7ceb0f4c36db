#!/bin/bash
# Round 4, session ZG: the live validator's n = 1 REF validate from cross-lane
# ballots (DC_LIVE_GATHER=1 build) -- live-path tests on it, then it alternated
# with the product (one-lane board assembly); then the round-end candidate
# (full GPU suite, smoke, bench, kernel trace).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
V=distributed-chess_amd/build/var/live1g
DCHESS_LIB=$PWD/$V/libdchess.so timeout -k 10 400 python -u -m pytest tests/test_gpu_live.py -x -v --timeout 120 --timeout-method thread > $O/pytest_live_zf.log 2>&1 || { tail -30 $O/pytest_live_zf.log; exit 1; }
tail -2 $O/pytest_live_zf.log
: > $O/live_gather_zf.txt
for r in 1 2 3; do
  echo "gather $(LD_LIBRARY_PATH=$V timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_gather_zf.txt || exit 2
  echo "assemble $(timeout -k 10 60 tools/latency_probe 5000)" >> $O/live_gather_zf.txt || exit 3
done
cat $O/live_gather_zf.txt

# then the round-end candidate
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_final.log 2>&1 || { tail -30 $O/pytest_gpu_final.log; exit 1; }
tail -2 $O/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.log 2>&1 || { cat $O/smoke_final.log; exit 2; }
cat $O/smoke_final.log
timeout -k 10 400 python -u bench.py > $O/bench_final.json 2> $O/bench_final.err || { tail -20 $O/bench_final.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_final.json'));print(d['value'],d['ms_per_step'])"
rm -rf $O/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_final -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_final.json 2> $O/prof_final.err || { tail -20 $O/prof_final.err; exit 4; }
echo prof ok
