#!/bin/bash
# A/B of the REF final stage (k_count2b vs k_count2c at several slot caps):
# parity tests first, then perft(7)/perft(6) bench lines per variant.
export TMPDIR=/tmp
# the knobs below exist only in the A/B build (make -C distributed-chess_amd ab)
export DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so
[ -f "$DCHESS_LIB" ] || { echo "build libdchess_ab.so first (make -C distributed-chess_amd ab)"; exit 3; }
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "perft or replica" > $O/ab_pytest.log 2>&1 || { tail -30 $O/ab_pytest.log; exit 1; }
tail -2 $O/ab_pytest.log
for v in ${AB_VARIANTS:-"DC_FINAL=2b" "DC_C2C_PHASE=3" "DC_C2C_PHASE=0"}; do
  env $v timeout -k 10 120 python -u bench.py --no-cpu --no-replay --steps 20 > $O/ab_$v.json 2> $O/ab_err.log || { cat $O/ab_err.log; exit 2; }
  python - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
print(sys.argv[1], "perft7 %.3e leaves/s  %.3f ms  count2 %.3f ms | perft6 %.3e" % (d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["perft6"]["value"]))
PY
done
