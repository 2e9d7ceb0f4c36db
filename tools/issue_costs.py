#!/usr/bin/env python3
"""gfx950 VALU issue costs per opcode from the dual_issue micro-benchmark's PMC
pass (tools/ubench/dual_issue.hip under rocprofv3 --pmc SQ_INSTS_VALU
SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE ...): SIMD cycles per wave64 instruction
at 1, 2, 4 and 8 waves per SIMD = kernel wall time x 2.4 GHz / (SQ_INSTS_VALU /
1024 SIMDs), cross-checked against GRBM_GUI_ACTIVE / 8 XCDs, and the fraction
of instructions issued in a dual-issue pair (2 x SQ_ACTIVE_INST_VALU2 /
SQ_INSTS_VALU).  Writes the cost table tools/bbprof.py model prices with.
  python tools/issue_costs.py PMC_CSV OUT.json"""
import csv
import json
import re
import sys

SRC = open(__file__.replace("issue_costs.py", "ubench/dual_issue.hip")).read()
NAMES = re.findall(r'"([^"]+)"', SRC[SRC.index("kName[] = {"):SRC.index("constexpr int kModes")])
# opcodes each micro-benchmark class stands for
OPS = {
    0: ["v_add_u32_e32"], 1: ["v_xor_b32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_xnor_b32_e32"],
    2: ["v_and_b32_e64", "v_or_b32_e64", "v_xor_b32_e64", "v_add_u32_e64"], 3: ["v_bitop3_b32"],
    4: ["v_bcnt_u32_b32"], 5: ["v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64"],
    6: ["v_lshlrev_b32_e32", "v_lshrrev_b32_e32", "v_ashrrev_i32_e32"], 7: ["v_cndmask_b32_e32"],
    8: ["v_cndmask_b32_e64"], 9: ["v_add3_u32"], 10: ["v_alignbit_b32"], 11: ["v_bfe_u32", "v_bfe_i32", "v_bfi_b32"],
    12: ["v_mov_b32_e32"], 13: ["v_ffbl_b32_e32", "v_ffbh_u32_e32"], 14: ["v_not_b32_e32"], 15: ["v_or3_b32"],
    16: ["v_lshl_or_b32"], 18: ["v_sub_u32_e32", "v_subrev_u32_e32"], 19: ["v_max_u32_e32", "v_min_u32_e32"],
    22: ["v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32"], 23: ["v_add_co_u32_e32", "v_addc_co_u32_e32"],
    24: ["v_lshl_add_u32"], 25: ["v_and_or_b32"], 26: ["v_perm_b32"], 27: ["v_mul_lo_u32"], 28: ["v_xad_u32"]}


def main():
    path, out = sys.argv[1], sys.argv[2]
    agg, order = {}, []
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("void k<"):
            continue
        key = (r["Dispatch_Id"], int(r["Kernel_Name"][7:r["Kernel_Name"].index(">")]), int(r["Grid_Size"]) // 65536)
        if key not in agg:
            agg[key] = {"t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
            order.append(key)
        agg[key][r["Counter_Name"]] = agg[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cls = {}
    for k in order:
        c = agg[k]
        _, m, w = k
        i = c["SQ_INSTS_VALU"] / 1024
        cls.setdefault(m, {"name": NAMES[m]})[str(w)] = {
            "cycles": round(c["t"] * 1e-9 * 2.4e9 / i, 3), "cycles_gui": round(c["GRBM_GUI_ACTIVE"] / 8 / i, 3),
            "paired_frac": round(2 * c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"], 3)}
    valu = {}
    for m, ops in OPS.items():
        if m in cls:
            for op in ops:
                valu[op] = {w: cls[m][w]["cycles_gui"] for w in ("1", "2", "4", "8")}
    slow = cls[4]  # v_bcnt: the single-issue class
    json.dump({"source": "tools/ubench/dual_issue.hip, rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU "
                         "SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE (profiles/r04/ubench_pmc.csv)",
               "unit": "SIMD cycles per wave64 instruction (GRBM_GUI_ACTIVE / 8 XCDs per SIMD instruction)",
               "classes": cls, "valu": valu,
               "valu_default": {w: slow[w]["cycles_gui"] for w in ("1", "2", "4", "8")},
               "valu_default_note": "opcodes the benchmark does not cover are priced as the single-issue class "
                                    "(v_bcnt_u32_b32)"}, open(out, "w"), indent=1)
    print(f"{len(valu)} opcodes priced; single-issue class {slow['4']['cycles_gui']} cycles at 4 waves/SIMD, "
          f"dual-issue class {cls[0]['4']['cycles_gui']}")


if __name__ == "__main__":
    main()
