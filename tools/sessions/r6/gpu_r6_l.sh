#!/bin/bash
# Round 6, session 3: FIDE final stage with 64-parent tail chunks
# (DC_C2B_GUIDED=1, product) against DC_C2B_GUIDED=0 (libdchess_old.so): FIDE
# parity tests on the product build, then alternating suite / FIDE perft(7) lines.
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
NEW=$PWD/distributed-chess_amd/libdchess.so EVEN=$PWD/distributed-chess_amd/libdchess_old.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_fide.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest_even.log 2>&1 || { tail -30 $O/pytest_even.log; exit 1; }
tail -2 $O/pytest_even.log
for v in guided old guided old guided old; do
  L=$NEW; [ $v = old ] && L=$EVEN
  DCHESS_LIB=$L timeout -k 10 200 python -u bench.py --only fidesuite,fide7 --steps 20 --no-cpu > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
  python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["fide_suite_d5"]; f = d["fide_perft7"]
print(sys.argv[2], "suite %.4f ms (final %.4f)  fide7 %.4f ms" % (s["ms_per_step"], s.get("final_kernel_ms", 0), f["ms_per_step"]))
PY
done
echo done
