#!/bin/bash
# Round 6, session 3: perft(6) (C2) steps over 2, 3 and 4 contexts
# (bench.py --perft-streams; default 3 at depth 6), the leg first in
# its process as in the default bench.
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
for r in 1 2 3; do
  for k in 2 3 4; do
    timeout -k 10 200 python -u bench.py --only perft6 --perft-streams $k --no-cpu > $O/b.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
    python - $O/b.json $k <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d["perft6"]; print("streams", sys.argv[2], "perft6 %.4f ms per step  %.3e leaves/s" % (p["ms_per_step"], p["value"]))
PY
  done
done
echo done
