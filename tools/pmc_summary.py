"""Aggregates rocprofv3 --pmc CSVs (gpurun_out/pmc_*) per kernel, averaged per
dispatch, and (with --json OUT --depth D --games N --plies P) writes the
roofline inputs bench.py reads from profiles/pmc_latest.json:
  hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B; the x2 is the
  gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md "HBM [CDNA4]"), and
  valu_lane_ops_per_unit = SQ_INSTS_VALU x 64 / units per dispatch."""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("root", nargs="?", default="gpurun_out")
ap.add_argument("--json")
ap.add_argument("--depth", type=int, default=7)
ap.add_argument("--replay-units", type=float, default=0.0, help="validated moves per replay dispatch")
ap.add_argument("--tx-units", type=float, default=0.0, help="transactions per k_verify_tx dispatch")
ap.add_argument("--source", default="")
a = ap.parse_args()
REF = {6: 120909581, 7: 3282734510}

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
meta = {}
for d in sorted(glob.glob(f"{a.root}/pmc_*")):
    for path in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add((d, r["Dispatch_Id"]))
            meta[k] = (r["VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"], r["Grid_Size"])
avg = {}
for k, cs in agg.items():
    avg[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    print(k, "vgpr/scratch/lds/grid", meta[k])
    print("   ", {c: round(v) for c, v in sorted(avg[k].items())})


def hbm(c):
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return None
    return (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024


if a.json:
    out = {}
    for k, c in avg.items():
        if "k_count2b<dc::RefRules" in k or "k_count2c<" in k:  # the REF final stage
            out[f"final_d{a.depth}"] = {"kernel": k, "hbm_bytes_per_launch": hbm(c),
                                          "valu_lane_ops_per_leaf": c.get("SQ_INSTS_VALU", 0) * 64 / REF[a.depth],
                                          "counters_per_dispatch": c, "source": a.source}
        if "k_replay_ref" in k and a.replay_units:
            out["replay"] = {"kernel": k, "hbm_bytes_per_launch": hbm(c),
                             "valu_lane_ops_per_move": c.get("SQ_INSTS_VALU", 0) * 64 / a.replay_units,
                             "counters_per_dispatch": c, "source": a.source}
        if "k_verify_tx" in k and a.tx_units:
            out["verify_tx"] = {"kernel": k, "hbm_bytes_per_launch": hbm(c),
                                "valu_lane_ops_per_unit": c.get("SQ_INSTS_VALU", 0) * 64 / a.tx_units,
                                "counters_per_dispatch": c, "source": a.source}
    json.dump(out, open(a.json, "w"), indent=1)
    print("wrote", a.json)
