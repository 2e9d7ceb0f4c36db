"""Aggregates rocprofv3 --pmc CSVs (ROOT/pmc_*/) per kernel, averaged per
dispatch, and (with --json OUT) writes the roofline inputs bench.py reads
from profiles/pmc_latest.json.

Per kernel record (units = the kernel's work units per dispatch, from --units):
  hbm_bytes_per_launch   = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B; the x2 is the
                           gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md
                           "HBM [CDNA4]")
  valu_lane_ops_per_unit = SQ_INSTS_VALU x 64 / units         (issue: full EXEC assumed)
  int_lane_ops_per_unit  = (SQ_INSTS_VALU_INT32 + _INT64) x 64 / units
                           (SURVEY §8d / BASELINE.md §3: the INT32 VALU fraction)
  valu_utilization       = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)
                           (rocprof's VALUUtilization: active lanes per VALU op)
  lds_conflict_per_lds_cycle = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  wait_frac              = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  dual_issue_frac        = 2 x SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU: the share of
                           VALU instructions issued in a same-quad-cycle pair
  valu_issue_slots_per_launch = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / 1024 SIMDs:
                           VALU issue slots (quad-cycles) one SIMD spends per
                           launch; x 4.34 cycles (the measured single-issue cost
                           at 4 waves/SIMD, profiles/r04/issue_costs.json) over the
                           kernel's cycles = the VALU issue-slot occupancy bench.py
                           reports.  (rocprof's VALUBusy is not used: its
                           SQ_ACTIVE_INST_VALU counts one quad-cycle per instruction,
                           so on gfx950 it is 2 x the issue fraction by construction.)
bench.py turns these into fractions of the 78.6 T lane-op/s issue peak with the
kernel's live HIP-event time.

--units takes KEY=PATTERN=UNITS triples, e.g. final_d7=k_count2c<=3282734510:
the first kernel whose name contains PATTERN (every '&'-separated part of it)
is written under KEY.
"""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("root", nargs="?", default="gpurun_out")
ap.add_argument("--json")
ap.add_argument("--units", action="append", default=[], help="KEY=PATTERN=UNITS per dispatch")
ap.add_argument("--source", default="")
a = ap.parse_args()

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
meta = {}
for d in sorted(glob.glob(f"{a.root}/pmc_*")):
    for path in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add((d, r["Dispatch_Id"]))
            meta[k] = {"vgpr": r["VGPR_Count"], "scratch": r["Scratch_Size"], "lds": r["LDS_Block_Size"],
                       "grid": r["Grid_Size"]}
avg = {}
for k, cs in agg.items():
    avg[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    print(k, meta[k])
    print("   ", {c: round(v) for c, v in sorted(avg[k].items())})


def derived(c, units):
    r = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        r["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    if units:
        if "SQ_INSTS_VALU" in c:
            r["valu_lane_ops_per_unit"] = c["SQ_INSTS_VALU"] * 64 / units
        if "SQ_INSTS_VALU_INT32" in c and "SQ_INSTS_VALU_INT64" in c:
            r["int_lane_ops_per_unit"] = (c["SQ_INSTS_VALU_INT32"] + c["SQ_INSTS_VALU_INT64"]) * 64 / units
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        r["valu_utilization"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)
    if c.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
        r["lds_conflict_per_lds_cycle"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"]
    if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in c:
        r["wait_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_INSTS_VALU") and "SQ_ACTIVE_INST_VALU2" in c:
        r["dual_issue_frac"] = 2 * c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"]
        r["valu_issue_slots_per_launch"] = (c["SQ_INSTS_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) / 1024
    if c.get("SQ_INSTS_VALU") and "SQ_INSTS_SALU" in c:
        r["salu_per_valu"] = c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"]
    return r


if a.json:
    out = {}
    for spec in a.units:
        key, pat, units = spec.split("=")
        for k, c in avg.items():
            if all(part in k for part in pat.split("&")):
                rec = {"kernel": k, "units_per_dispatch": float(units), "counters_per_dispatch": c,
                       "resources": meta[k], "source": a.source}
                rec.update(derived(c, float(units)))
                # legacy names bench.py reads
                if "valu_lane_ops_per_unit" in rec:
                    rec["valu_lane_ops_per_leaf"] = rec["valu_lane_ops_per_move"] = rec["valu_lane_ops_per_unit"]
                out[key] = rec
                break
    json.dump(out, open(a.json, "w"), indent=1)
    print("wrote", a.json)
    for key, rec in out.items():
        print(key, {x: (round(v, 4) if isinstance(v, float) else v) for x, v in rec.items()
                    if x not in ("counters_per_dispatch", "resources", "source", "kernel")})
