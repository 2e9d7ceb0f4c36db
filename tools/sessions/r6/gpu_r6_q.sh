#!/bin/bash
# Round 6, session 3: the suite batch over 2 and 4 contexts inside longer
# bench runs (the default bench gave 0.332 ms on 4 where --only fidesuite
# --suite-batch-only gave 0.297-0.300).
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
for legs in "fidesuite" "perft6,fide7,fidesuite"; do
  for k in 2 4; do
    timeout -k 10 300 python -u bench.py --only $legs --perft-streams $k --no-cpu > $O/b.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
    python - $O/b.json "$legs" $k <<'PY'
import json, sys
s = json.load(open(sys.argv[1]))["fide_suite_d5"]
print(sys.argv[2], "streams", sys.argv[3], "suite %.4f ms per step (final %.4f)" % (s["ms_per_step"], s.get("final_kernel_ms", 0)))
PY
  done
done
echo done
