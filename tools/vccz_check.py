#!/usr/bin/env python3
"""Static check for the round-5 fault shape, on compiler
assembly (.s) or on the disassembly of a built library's code objects.

The round-4 reproducer (k_count2b<FideRules, 1> with the kAtt king set) loses
leaves only when a wave of another workgroup on the same SIMD issues
single-issue VALU instructions; raising the victim wave's priority (s_setprio 3)
over exactly two instructions removes the fault (profiles/r05/fault_study.md):

    v_cmp_ne_u64_e32 vcc, 0, v[102:103]      a __ballot line gate of analyse
    v_lshlrev_b64 v[106:107], v135, -2       above_mask(ksq)      <- window
    v_lshlrev_b64 v[102:103], v135, -1       below_mask(ksq): overwrites the
    s_cbranch_vccz .LBB40_24                 compare's operands    <- window

The shape flagged here: a VCCZ branch (s_cbranch_vccz / vccnz) whose VCC comes
from a VALU compare whose source VGPRs are overwritten by a 64-bit shift
(v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) between the compare and the
branch.  --any widens it to any VALU write of the compare's sources (common
register reuse the compiler emits everywhere; reported, not failed).  (It is the window the priority
experiment isolated, not a proven sufficient condition: the shipped FIDE
kernels carried the same sequence and passed the co-residency stress test;
they no longer carry it, dc_fide_rules.h analyse.)

usage: vccz_check.py FILE.s|LIB.so [--strict] [--any] [kernel-substring ...]
--strict: exit 1 if any kernel has the shape."""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scratch_bounds_check import kernels_from_lib, kernels_from_s  # noqa: E402

VCC_WRITER = re.compile(r"^(v_cmpx?_\w+_e32\s+vcc|v_\w+_co_u32_e32\b|v_(addc|subb|subbrev)_co_u32_e32\b|s_\w+\s+vcc\b|"
                        r"v_\w+\s+vcc\b)")
BR = re.compile(r"^s_cbranch_vccn?z\b")


def vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def insts(lines):
    out = []
    for ln in lines:
        s = ln.split(";")[0].split("//")[0].strip()
        if s and not s.startswith(".") and not s.endswith(":"):
            out.append(s)
    return out


SHIFT64 = re.compile(r"^v_(lshlrev|lshrrev|ashrrev)_[bi]64\b")


def shape(lines, lookback=8, any_writer=False):
    """[(compare, [instructions up to the branch])] of flagged VCCZ branches."""
    ins = insts(lines)
    hits = []
    for i, s in enumerate(ins):
        if not BR.match(s):
            continue
        for j in range(i - 1, max(-1, i - lookback), -1):
            if not VCC_WRITER.match(ins[j]):
                continue
            if ins[j].startswith("v_cmp"):
                args = [a.strip() for a in ins[j].split(None, 1)[1].split(",")]
                src = set().union(*[vregs(a) for a in args[1:]])
                written = set()
                for k in range(j + 1, i):
                    p = ins[k].split(None, 1)
                    if p[0].startswith("v_") and len(p) > 1 and (any_writer or SHIFT64.match(ins[k])):
                        written |= vregs(p[1].split(",")[0].strip())
                if src & written:
                    hits.append((ins[j], ins[j + 1:i + 1]))
            break
    return hits


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    strict = "--strict" in sys.argv
    any_writer = "--any" in sys.argv
    path, subs = args[0], args[1:]
    ks = kernels_from_lib(path) if path.endswith(".so") else kernels_from_s(path)
    bad = 0
    for name, (lines, _, _) in sorted(ks.items()):
        if subs and not any(x in name for x in subs):
            continue
        h = shape(lines, any_writer=any_writer)
        if h:
            bad += 1
            print(f"{name}: {len(h)}  e.g. {h[0][0]} | {' ; '.join(h[0][1])}")
    print(f"{bad} of {len(ks)} kernels have the shape")
    sys.exit(1 if strict and bad else 0)


if __name__ == "__main__":
    main()
