#!/bin/bash
# PMC passes over the state-hash kernel (tools/time_hash.py), one rocprofv3 run per pass.
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; rm -rf $O/hpmc_*
pass() { GAMES=${GAMES:-200000} timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d $O/hpmc_$2 -o p -- python3 tools/time_hash.py > /dev/null 2>> $O/hpmc.err; }
pass "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" a && \
pass "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" b && \
pass "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" c && pass "VALUUtilization" d || { tail $O/hpmc.err; exit 5; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/hpmc_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "state_hash" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(agg.items()):
    print(f"   {c:28s} {sum(v)/len(v):.4g}")
PY
