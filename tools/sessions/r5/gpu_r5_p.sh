#!/bin/bash
# Round-5 session P: the FIDE split-pass probe (ADVICE), the FIDE suite after
# the C2bShared change, and the bench's batched suite leg with its kernel trace.
O=gpurun_out/r5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fide_split.py tests/test_gpu_fide.py > $O/pytest_p.log 2>&1 || { tail -30 $O/pytest_p.log; exit 1; }
tail -3 $O/pytest_p.log
timeout -k 10 300 python -u bench.py --only fidesuite,fide7 --no-cpu > $O/bench_p.json 2> $O/bench_p.err || { tail -20 $O/bench_p.err; exit 1; }
cat $O/bench_p.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_p -o fs -- python3 bench.py --only fidesuite --no-cpu --profile-only > $O/prof_p.log 2>&1 || { tail -20 $O/prof_p.log; exit 1; }
find $O/prof_p -name "*kernel_stats.csv" | head -3
