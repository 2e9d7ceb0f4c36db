#!/bin/bash
# LDS / issue counters of the replay kernel alone (bench.py --only replay), one
# rocprofv3 --pmc pass per counter set; summary per kernel -> gpurun_out/pmc_replay.txt
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
P="--steps 1 --warmup 0 --no-cpu --only replay --replay-steps 2"
i=0
for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           ${EXTRA_CNT}; do
  i=$((i+1)); rm -rf $O/pmcr_$i
  timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d $O/pmcr_$i -o p -- python bench.py $P > /dev/null 2>> $O/pmcr_err.log || { tail -20 $O/pmcr_err.log; exit 2; }
done
python - <<'PY' | tee $O/pmc_replay.txt
import csv, glob
from collections import defaultdict
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob("gpurun_out/pmcr_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "replay" in k or "gen_games" in k:
            per[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, c in per.items():
    print(k, {n: f"{sum(d.values()) / len(d):.4g}" for n, d in sorted(c.items())})
PY
