#!/bin/bash
# Round-5 session Q: the REF target-side pawn correction (DC_C2C_GCORR) against
# the REF goldens, then the FIDE split-pass probe and suite (session P), and the
# bench's perft / FIDE legs with a kernel trace.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref.py tests/test_gpu_dfs.py tests/test_gpu_fide_split.py tests/test_gpu_fide.py > $O/pytest_q.log 2>&1 || { tail -30 $O/pytest_q.log; exit 1; }
tail -3 $O/pytest_q.log
timeout -k 10 300 python -u bench.py --only perft,perft6,perft8,fidesuite,fide7 --no-cpu > $O/bench_q.json 2> $O/bench_q.err || { tail -20 $O/bench_q.err; exit 1; }
cat $O/bench_q.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_q -o q --output-format csv -- python3 bench.py --only perft,fidesuite --no-cpu --profile-only > $O/prof_q.log 2>&1 || { tail -20 $O/prof_q.log; exit 1; }
find $O/prof_q -name "*kernel_stats.csv" -exec head -12 {} \;
