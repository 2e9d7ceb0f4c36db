#!/bin/bash
# Round-4 session Y: the full GPU suite, smoke() and the bench of the
# current product (the round-end candidate).
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_y.log 2>&1 || { tail -30 $O/pytest_gpu_y.log; exit 1; }
tail -2 $O/pytest_gpu_y.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_y.log 2>&1 || { cat $O/smoke_y.log; exit 2; }
cat $O/smoke_y.log
timeout -k 10 400 python -u bench.py > $O/bench_y.json 2> $O/bench_y.err || { tail -20 $O/bench_y.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_y.json'));print(d['value'],d['ms_per_step'])"
