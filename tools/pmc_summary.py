"""Aggregates rocprofv3 --pmc CSVs (gpurun_out/pmc_*) per kernel, averaged per dispatch."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
meta = {}
for d in sorted(glob.glob(f"{root}/pmc_*")):
    for r in csv.DictReader(open(d + "/p_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
        meta[k] = (r["VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"], r["Grid_Size"])
for k, cs in agg.items():
    out = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    print(k, "vgpr/scratch/lds/grid", meta[k])
    print("   ", {c: round(v) for c, v in sorted(out.items())})
