#!/bin/bash
# Round 6, session 3: FIDE final stage chunking A/B (DC_C2B_EVEN=1 in
# libdchess_even.so against the product build): FIDE parity tests on the
# variant, then alternating suite bench lines.
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
NEW=$PWD/distributed-chess_amd/libdchess.so EVEN=$PWD/distributed-chess_amd/libdchess_even.so
DCHESS_LIB=$EVEN timeout -k 10 400 python -u -m pytest tests/test_gpu_fide.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest_even.log 2>&1 || { tail -30 $O/pytest_even.log; exit 1; }
tail -2 $O/pytest_even.log
for v in base even base even base even; do
  L=$NEW; [ $v = even ] && L=$EVEN
  DCHESS_LIB=$L timeout -k 10 200 python -u bench.py --only fidesuite,fide7 --steps 20 --no-cpu > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
  python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["fide_suite_d5"]; f = d["fide_perft7"]
print(sys.argv[2], "suite %.4f ms (final %.4f)  fide7 %.4f ms" % (s["ms_per_step"], s.get("final_kernel_ms", 0), f["ms_per_step"]))
PY
done
echo done
