#!/bin/bash
# Round 6, session 3: state hash time against batch size around whole rounds of
# resident lanes (196,608 = 256 CUs x 3 blocks x 256 threads): 5.00, 5.09, 6.00 rounds.
export TMPDIR=/tmp
O=gpurun_out/r6ah; mkdir -p $O
for rep in 1 2; do
for n in 983040 1000000 1179648; do
  timeout -k 10 200 python -u bench.py --only hash --hash-steps 5 --hash-games $n --no-cpu > $O/bench_$n.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
  python - $O/bench_$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["state_hash"]; n = int(sys.argv[2])
print(n, "games (%.2f rounds): call %.3f ms, kernel %.4f ms, kernel per 1M games %.4f ms" % (n / 196608, d["ms_per_step"], d["kernel_avg_ms"], d["kernel_avg_ms"] * 1e6 / n))
PY
done
done
echo done
