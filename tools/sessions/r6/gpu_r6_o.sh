#!/bin/bash
# Round 6, session 3: the FIDE suite batch's step over 2, 3 and 4 contexts
# (bench.py --perft-streams; the default is 2).
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
for r in 1 2; do
  for k in 2 3 4; do
    timeout -k 10 200 python -u bench.py --only fidesuite --suite-batch-only --perft-streams $k --steps 24 --no-cpu > $O/bench_$k.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
    python - $O/bench_$k.json $k <<'PY'
import json, sys
s = json.load(open(sys.argv[1]))["fide_suite_d5"]
print("streams", sys.argv[2], "suite %.4f ms per step (final %.4f)" % (s["ms_per_step"], s.get("final_kernel_ms", 0)))
PY
  done
done
echo done
