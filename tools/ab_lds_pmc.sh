#!/bin/bash
# LDS counters of k_count3c for the product library and a variant (A/B build by hand:
# distributed-chess_amd/build/var/lib_$V.so), one rocprofv3 --pmc pass each.
export TMPDIR=/tmp
V=${V:-soa}
for v in prod $V; do
  L=$PWD/distributed-chess_amd/build/var/lib_$v.so; [ $v = prod ] && L=$PWD/distributed-chess_amd/libdchess.so
  rm -rf gpurun_out/lds_$v
  DCHESS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/lds_$v -o p -- python bench.py --only perft --no-cpu --steps 4 --warmup 1 > /dev/null 2>> gpurun_out/lds_err.log || { tail -5 gpurun_out/lds_err.log; exit 1; }
  python - "$v" <<'PY'
import csv, glob, sys
from collections import defaultdict
v = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in glob.glob(f"gpurun_out/lds_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_count3c<0" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
print(v, {k: f"{sum(d.values()) / len(d):.4g}" for k, d in sorted(acc.items())})
PY
done
