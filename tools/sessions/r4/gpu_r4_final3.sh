#!/bin/bash
# Round-4 session FINAL3 (last tree): the full GPU suite, smoke() and the bench of the
# current product (the round-end candidate).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_final3.log 2>&1 || { tail -30 $O/pytest_gpu_final3.log; exit 1; }
tail -2 $O/pytest_gpu_final3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final3.log 2>&1 || { cat $O/smoke_final3.log; exit 2; }
cat $O/smoke_final3.log
timeout -k 10 400 python -u bench.py > $O/bench_final3.json 2> $O/bench_final3.err || { tail -20 $O/bench_final3.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_final3.json'));print(d['value'],d['ms_per_step'])"
rm -rf $O/prof_final3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_final3 -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof_final32.json 2> $O/prof_final32.err || { tail -20 $O/prof_final32.err; exit 4; }
echo prof ok
