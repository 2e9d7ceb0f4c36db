#!/bin/bash
# Round 6, session 3, final tree: the whole GPU suite, smoke, the default
# bench and its rocprofv3 kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -30 $O/pytest_gpu_full.log; exit 11; }
tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 12; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 13; }
cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 14; }
echo done
