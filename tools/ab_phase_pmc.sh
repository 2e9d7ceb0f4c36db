#!/bin/bash
# SQ counters of k_count2c per DC_C2C_PHASE variant (A/B build): the VALU / LDS
# instruction cost of each part of the final stage (phases 1/2/5/6 skip work
# and give wrong counts: instruction accounting only).  One rocprofv3 --pmc
# pass per variant, perft(startpos, 7) x 3.
export TMPDIR=/tmp
export DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so
[ -f "$DCHESS_LIB" ] || { echo "build libdchess_ab.so first (make -C distributed-chess_amd ab)"; exit 3; }
O=gpurun_out; mkdir -p $O
CNT=${CNT:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"}
for p in ${PHASES:-0 1 2 5 6}; do
  DC_C2C_PHASE=$p RUNS=3 timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d $O/abpmc_$p -o p -- python tools/time_final.py > $O/abpmc_$p.txt 2> $O/abpmc_err.log || { tail -20 $O/abpmc_err.log; exit 2; }
done
python - ${PHASES:-0 1 2 5 6} <<'PY'
import csv, glob, sys
from collections import defaultdict
for p in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/abpmc_{p}/**/*counter_collection.csv", recursive=True)
    per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for r in csv.DictReader(open(f[0])):
        if "k_count2c" in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    avg = {k: sum(d.values()) / len(d) for k, d in per.items()}
    print(p, {k: f"{v:.4g}" for k, v in sorted(avg.items())}, open(f"gpurun_out/abpmc_{p}.txt").read().strip(), flush=True)
PY
