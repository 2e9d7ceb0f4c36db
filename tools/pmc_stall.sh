#!/bin/bash
# Stall-reason PMC passes for the perft final stage (one rocprofv3 run per pass).
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; rm -rf $O/stall_*
P="${STALL_ARGS:---steps 3 --warmup 1 --no-cpu --profile-only --no-replay} ${BENCH_ARGS}"
pass() { local c=$1 t=$2; timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/stall_$t -o p -- python bench.py $P > /dev/null 2>> $O/stall.err; }
pass "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES" a && \
pass "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT" b && \
pass "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" c && pass "VALUUtilization" d && pass "FETCH_SIZE" e || { tail $O/stall.err; exit 5; }
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/stall_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "count2" in k or "count3" in k or "replay" in k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}")
PY
