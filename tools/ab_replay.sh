#!/bin/bash
# A/B of the REF replay kernel (DC_REPLAY=1: arithmetic k_replay_ref; =3: k_replay_ref3;
# default: k_replay_ref4): replay parity tests, then replay bench lines.
export TMPDIR=/tmp
# the knobs below exist only in the A/B build (make -C distributed-chess_amd ab)
export DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so
[ -f "$DCHESS_LIB" ] || { echo "build libdchess_ab.so first (make -C distributed-chess_amd ab)"; exit 3; }
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "replay or gen or apply or validate or smoke" > $O/abr_pytest.log 2>&1 || { tail -30 $O/abr_pytest.log; exit 1; }
tail -2 $O/abr_pytest.log
for v in ${AB_VARIANTS:-"DC_REPLAY=3" "DC_REPLAY=4"}; do
  env ${v//,/ } timeout -k 10 120 python -u bench.py --only replay --replay-steps 10 > $O/abr_$v.json 2> $O/abr_err.log || { cat $O/abr_err.log; exit 2; }
  python - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/abr_{sys.argv[1]}.json"))["replay"]
print(sys.argv[1], "replay %.3e moves/s  %.3f ms  kernel %.3f ms  parity %s" % (d["value"], d["ms_per_step"], d["kernel_avg_ms"], d["replay_parity"]))
PY
done
