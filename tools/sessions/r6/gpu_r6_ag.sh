#!/bin/bash
# Round 6, session 3: global pieces (names, start history) copied 8 loads at a time (DC_HASH_GLB8=1, libdchess.so) against a load and wait a byte (libdchess_old.so).
# hash/replay-info parity, then alternating bench lines.
export TMPDIR=/tmp
O=gpurun_out/r6ag; mkdir -p $O
NEW=$PWD/distributed-chess_amd/libdchess.so OLD=$PWD/distributed-chess_amd/libdchess_old.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "hash or info or replay" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old new old new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  DCHESS_LIB=$L timeout -k 10 200 python -u bench.py --only hash --hash-steps 5 --no-cpu > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
  python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["state_hash"]
print(sys.argv[2], "hash %.3f ms per call  %.3e hashes/s  kernels %s" % (d["ms_per_step"], d["value"], {k: round(d[k], 4) for k in ("kernel_avg_ms", "replay_prepass_ms")}))
PY
done
echo done
