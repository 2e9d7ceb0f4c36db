#!/bin/bash
# Round 6, session 3: generator table reads batched ahead of the slot counts
# (DC_GEN_BATCH=1, product) A/B against the old form (libdchess_old.so:
# DC_GEN_BATCH=0 DC_GEN_NOBR=0).  Every GPU step has its own limit; the first failure ends it.
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
NEW=$PWD/distributed-chess_amd/libdchess.so OLD=$PWD/distributed-chess_amd/libdchess_old.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "gen or replay" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  DCHESS_LIB=$L timeout -k 10 200 python -u bench.py --only replay --replay-steps 5 --no-cpu > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
  python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("replay", d)
e = r["end_to_end"]
print(sys.argv[2], "gen %.3f ms  e2e %.3e  replay kernel %.3f ms parity %s" % (e["gen_kernel_avg_ms"], e["value"], r["kernel_avg_ms"], r.get("replay_parity")))
PY
done
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  DCHESS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/pmc_gen_$v -o p -- python bench.py --only replay --replay-steps 1 --no-cpu > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 3; }
done
echo done
