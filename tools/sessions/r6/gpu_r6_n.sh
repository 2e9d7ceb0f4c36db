#!/bin/bash
# Round 6, session 3: Keccak-f round loop unrolled 2 and 4 times
# (DC_KECCAK_UNROLL, libdchess_ku2/ku4.so) against the product (1): the hash
# tests on each variant, then alternating state-hash bench lines.
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
P=$PWD/distributed-chess_amd
for v in ku2 ku4; do
  DCHESS_LIB=$P/libdchess_$v.so timeout -k 10 300 python -u -m pytest tests/test_statehash.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for r in 1 2 3; do
  for v in base ku2 ku4; do
    L=$P/libdchess.so; [ $v != base ] && L=$P/libdchess_$v.so
    DCHESS_LIB=$L timeout -k 10 200 python -u bench.py --only hash --hash-steps 5 --no-cpu > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
    python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["state_hash"]
print(sys.argv[2], "hash %.3f ms per call  kernel %.4f ms" % (d["ms_per_step"], d["kernel_avg_ms"]))
PY
  done
done
echo done
