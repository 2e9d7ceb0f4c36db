#!/bin/bash
# Round 6, session 3: the suite batch on four contexts after the perft legs,
# with the shared contexts (as the bench) and with contexts of its own
# (DC_SUITE_FRESH=1).
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
for r in 1 2; do
  for fresh in 0 1; do
    for k in 2 4; do
      DC_SUITE_FRESH=$([ $fresh = 1 ] && echo 1) timeout -k 10 300 python -u bench.py --only perft6,fide7,fidesuite --perft-streams $k --no-cpu > $O/b.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
      python - $O/b.json $fresh $k <<'PY'
import json, sys
s = json.load(open(sys.argv[1]))["fide_suite_d5"]
print("fresh", sys.argv[2], "streams", sys.argv[3], "suite %.4f ms per step (final %.4f)" % (s["ms_per_step"], s.get("final_kernel_ms", 0)))
PY
    done
  done
done
echo done
