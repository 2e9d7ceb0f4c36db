#!/usr/bin/env python3
"""bbprof.py -- exact basic-block execution counts of one gfx950 kernel, and the
instruction-mix cycle model built on them.  Measurement tooling only: the
product never loads an instrumented build.

Subcommands
  instrument IN.s OUT.s --kernel SUBSTR --sym NAME
      Copies the device assembly, inserting at the start of every basic block of
      the first kernel whose symbol contains SUBSTR a per-wave counter
      increment, and before every s_endpgm a flush of the wave's counters into
      the __device__ array NAME (u64[8192], DC_BBPROF_DEFINE in dc_kernels.h).
      A counter is one lane of a reserved VGPR above the kernel's own registers
      (v_readlane / s_add_u32 / v_writelane: EXEC-independent, so a block that
      a wave runs with EXEC = 0 is counted too -- it still pays the issue
      cycles).  SCC is saved and restored around the add.  The kernel's own
      instructions, registers and order are untouched; the descriptor's VGPR /
      SGPR counts grow by the reserved registers.
  blocks IN.s --kernel SUBSTR [--json OUT]
      The kernel's basic blocks with their static instruction classes (the
      block numbering matches `instrument`).
  lines IN_G.s --kernel SUBSTR --counts COUNTS.json --costs COSTS.json [--orig ORIG.s]
      Per source line: the VALU issue cycles, instructions and the single-issue
      share, from an assembly of the same build compiled with
      -g -gline-tables-only (the .loc comments; the innermost inlined
      location).  --orig checks that its blocks match the counted build's.
  model IN.s --kernel SUBSTR --counts COUNTS.json [--costs COSTS.json] [--pmc PMC.json]
      Dynamic instruction counts = sum over blocks of executions x static
      instructions; the VALU mix by issue class; predicted SIMD cycles from the
      measured per-class issue costs (tools/ubench/dual_issue.hip); checked
      against rocprofv3's SQ_INSTS_VALU / SALU / LDS of the same kernel.

The block numbering is the order of block starts in the function: block 0 at
the entry, then every `.LBB` label and every `; %bb.N:` fall-through marker.
"""
import argparse
import collections
import json
import re
import sys

LABEL = re.compile(r"^(\.LBB\d+_\d+):")
BBCOMMENT = re.compile(r"^; %bb\.\d+:")
INSTR = re.compile(r"^\s+([a-z_][a-z0-9_]*)(\s|$)")


def find_kernel(lines, substr):
    """(start, end) line indices of the kernel body: from its label to .Lfunc_end."""
    start = None
    for i, ln in enumerate(lines):
        if start is None:
            if ln.startswith("_Z") and ln.split(":")[0].find(substr) >= 0 and ":" in ln and not ln.startswith("\t"):
                start = i
        elif ln.startswith(".Lfunc_end"):
            return start, i
    raise SystemExit(f"kernel containing {substr!r} not found")


def kernel_name(lines, start):
    return lines[start].split(":")[0]


def is_instr(ln):
    m = INSTR.match(ln)
    if not m:
        return None
    op = m.group(1)
    if op.startswith("."):
        return None
    return op


def split_blocks(lines, start, end):
    """[(first_line, [(line_no, opcode, text), ...]), ...] in order."""
    blocks = []
    cur = [start + 1, []]
    for i in range(start + 1, end):
        ln = lines[i]
        if LABEL.match(ln) or BBCOMMENT.match(ln):
            if cur[1] or blocks or cur[0] != start + 1:
                blocks.append(cur)
            cur = [i + 1, []]
            continue
        op = is_instr(ln)
        if op:
            cur[1].append((i, op, ln.strip()))
    blocks.append(cur)
    # drop an empty leading block (label right after the function label)
    return [b for b in blocks if b[1] or b is blocks[0]]


# ------------------------------------------------------------ classification
def classify(op, text):
    """Issue class of one instruction."""
    if op.startswith("s_"):
        if op in ("s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_sleep", "s_setprio", "s_trap"):
            return "s_ctrl"
        if op.startswith("s_cbranch") or op == "s_branch":
            return "branch"
        if op.startswith("s_load") or op.startswith("s_buffer_load") or op in ("s_memtime", "s_memrealtime", "s_dcache_inv"):
            return "smem"
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu:" + op
    return "other:" + op


def valu_key(op, text):
    """Cost key of a VALU instruction: the opcode with its encoding suffix."""
    return op


def static_mix(blocks):
    mix = []
    for first, ins in blocks:
        c = collections.Counter()
        for _, op, text in ins:
            c[classify(op, text)] += 1
        mix.append(c)
    return mix


# ------------------------------------------------------------- instrumenting
VREG = re.compile(r"\bv\[?(\d+)(?::(\d+))?\]?")
SREG = re.compile(r"\bs\[?(\d+)(?::(\d+))?\]?")


def max_reg(lines, start, end, rx):
    hi = -1
    for i in range(start, end):
        ln = lines[i]
        if not is_instr(ln):
            continue
        body = ln.split(";")[0]
        for m in rx.finditer(body):
            a = int(m.group(1))
            b = int(m.group(2)) if m.group(2) else a
            hi = max(hi, a, b)
    return hi


def instrument(args):
    lines = open(args.inp).read().split("\n")
    start, end = find_kernel(lines, args.kernel)
    name = kernel_name(lines, start)
    blocks = split_blocks(lines, start, end)
    nb = len(blocks)
    if nb > 8 * 64 * 4:
        raise SystemExit(f"{nb} blocks: more than the counter VGPRs hold")
    # descriptor fields
    desc = {}
    dstart = None
    for i in range(start, len(lines)):
        if lines[i].strip().startswith(".amdhsa_kernel " + name):
            dstart = i
        if dstart is not None:
            m = re.match(r"\s*(\.amdhsa_\w+)\s+(\S+)", lines[i])
            if m:
                desc[m.group(1)] = (i, m.group(2))
            if lines[i].strip() == ".end_amdhsa_kernel":
                break
    nv = int(desc[".amdhsa_next_free_vgpr"][1])
    acc = int(desc[".amdhsa_accum_offset"][1])
    used_v = max_reg(lines, start, end, VREG) + 1
    used_s = max_reg(lines, start, end, SREG) + 1
    if used_v > acc:
        raise SystemExit("kernel uses AGPRs or VGPRs past accum_offset: not handled")
    n_ctr = (nb + 63) // 64
    vbase = (acc + 3) // 4 * 4
    vaddr = vbase + n_ctr  # flush: address, then the (value, 0) pair at an even vdata
    vdata = (vaddr + 2) // 2 * 2
    new_nv = vdata + 2
    if new_nv > 256:
        raise SystemExit("not enough VGPRs for the counters")
    sp = (max(used_s, int(desc[".amdhsa_next_free_sgpr"][1])) + 1) // 2 * 2  # even pair sT, sS
    if sp + 2 > 102:
        raise SystemExit("not enough SGPRs")
    sT, sS = sp, sp + 1
    out = lines[:]
    inserts = collections.defaultdict(list)  # line index -> list of lines inserted BEFORE it

    def bump(k):
        v, lane = vbase + k // 64, k % 64
        return [f"\ts_cselect_b32 s{sS}, 1, 0\t; bbprof {k}",
                "\ts_nop 1",
                f"\tv_readlane_b32 s{sT}, v{v}, {lane}",
                "\ts_nop 4",
                f"\ts_add_u32 s{sT}, s{sT}, 1",
                f"\tv_writelane_b32 v{v}, s{sT}, {lane}",
                f"\ts_cmp_lg_u32 s{sS}, 0"]

    # zero the counters at entry (EXEC is the launched lanes at entry: use
    # v_writelane-free zeroing with exec forced, restored after)
    entry = blocks[0][1][0][0]
    zero = [f"\ts_mov_b64 s[{sT}:{sS}], exec\t; bbprof entry", "\ts_mov_b64 exec, -1"]
    zero += [f"\tv_mov_b32 v{vbase + i}, 0" for i in range(n_ctr)]
    zero += [f"\ts_mov_b64 exec, s[{sT}:{sS}]"]
    inserts[entry] += zero
    for k, (first, ins) in enumerate(blocks):
        if not ins:
            continue
        at = ins[0][0]
        inserts[at] += bump(k)
    # flush before every s_endpgm
    for i in range(start, end):
        if is_instr(lines[i]) == "s_endpgm":
            fl = ["\ts_mov_b64 exec, -1\t; bbprof flush",
                  f"\tv_mbcnt_lo_u32_b32 v{vaddr}, -1, 0",
                  f"\tv_mbcnt_hi_u32_b32 v{vaddr}, -1, v{vaddr}",
                  f"\tv_lshlrev_b32_e32 v{vaddr}, 3, v{vaddr}",
                  f"\ts_getpc_b64 s[{sT}:{sS}]",
                  f"\ts_add_u32 s{sT}, s{sT}, {args.sym}@rel32@lo+4",
                  f"\ts_addc_u32 s{sS}, s{sS}, {args.sym}@rel32@hi+12",
                  f"\tv_mov_b32 v{vdata + 1}, 0"]
            for c in range(n_ctr):
                fl += [f"\tv_mov_b32 v{vdata}, v{vbase + c}",
                       f"\tglobal_atomic_add_x2 v{vaddr}, v[{vdata}:{vdata + 1}], s[{sT}:{sS}]",
                       f"\tv_add_u32_e32 v{vaddr}, 0x200, v{vaddr}"]
            fl += ["\ts_waitcnt vmcnt(0)"]
            inserts[i] += fl
    res = []
    for i, ln in enumerate(out):
        if i in inserts:
            res.extend(inserts[i])
        res.append(ln)
    # descriptor / metadata
    text = "\n".join(res)
    acc_new = (new_nv + 3) // 4 * 4

    def setfield(t, field, val):
        return re.sub(r"(\.amdhsa_kernel " + re.escape(name) + r"\n(?:.*\n)*?\s*" + re.escape(field) + r"\s+)\d+",
                      lambda m: m.group(1) + str(val), t, count=1)

    text = setfield(text, ".amdhsa_next_free_vgpr", acc_new)
    text = setfield(text, ".amdhsa_accum_offset", acc_new)
    text = setfield(text, ".amdhsa_next_free_sgpr", max(sp + 2, int(desc[".amdhsa_next_free_sgpr"][1])))
    text = re.sub(re.escape(name) + r"\.num_vgpr, \d+", f"{name}.num_vgpr, {acc_new}", text)
    text = re.sub(re.escape(name) + r"\.numbered_sgpr, \d+", f"{name}.numbered_sgpr, {sp + 2}", text)
    # code-object metadata (the runtime's occupancy queries read it)
    mi = text.find(".name:           " + name + "\n")
    if mi >= 0:
        seg_end = text.find(".wavefront_size", mi)
        seg = text[mi:seg_end]
        seg = re.sub(r"\.vgpr_count:\s+\d+", f".vgpr_count:     {acc_new}", seg)
        seg = re.sub(r"\.sgpr_count:\s+\d+", lambda m: m.group(0), seg)
        text = text[:mi] + seg + text[seg_end:]
    open(args.out, "w").write(text)
    json.dump({"kernel": name, "blocks": nb, "counter_vgprs": [vbase, vbase + n_ctr - 1], "sgprs": [sT, sS],
               "vgpr_before": nv, "vgpr_after": acc_new}, open(args.out + ".json", "w"), indent=1)
    print(f"{name}: {nb} blocks instrumented, VGPRs {nv} -> {acc_new}, SGPR pair s[{sT}:{sS}]", file=sys.stderr)


# ------------------------------------------------------------------ reporting
def load_blocks(path, kernel):
    lines = open(path).read().split("\n")
    start, end = find_kernel(lines, kernel)
    return kernel_name(lines, start), split_blocks(lines, start, end)


def blocks_cmd(args):
    name, blocks = load_blocks(args.inp, args.kernel)
    mix = static_mix(blocks)
    rec = []
    for k, ((first, ins), c) in enumerate(zip(blocks, mix)):
        valu = sum(v for x, v in c.items() if x.startswith("valu:"))
        rec.append({"block": k, "line": first, "n": len(ins), "valu": valu, "salu": c["salu"], "lds": c["lds"],
                    "vmem": c["vmem"], "branch": c["branch"]})
    if args.json:
        json.dump({"kernel": name, "blocks": rec}, open(args.json, "w"), indent=1)
    print(name, len(blocks), "blocks")
    for r in rec:
        print(r)


def model_cmd(args):
    name, blocks = load_blocks(args.inp, args.kernel)
    counts = json.load(open(args.counts))
    per_block = counts["wave_executions"]
    if len(per_block) < len(blocks):
        raise SystemExit(f"counts for {len(per_block)} blocks, kernel has {len(blocks)}")
    dyn = collections.Counter()
    hot = []
    for k, (first, ins) in enumerate(blocks):
        e = per_block[k]
        if not e:
            continue
        c = collections.Counter(classify(op, t) for _, op, t in ins)
        for x, v in c.items():
            dyn[x] += v * e
        hot.append((e * sum(v for x, v in c.items() if x.startswith("valu:")), k, e, len(ins)))
    valu = {x[5:]: v for x, v in dyn.items() if x.startswith("valu:")}
    n_valu = sum(valu.values())
    out = {"kernel": name, "launches": counts.get("launches", 1), "valu": n_valu, "salu": dyn["salu"],
           "lds": dyn["lds"], "vmem": dyn["vmem"], "smem": dyn["smem"], "branch": dyn["branch"],
           "s_ctrl": dyn["s_ctrl"]}
    L = max(1, out["launches"])
    for k in ("valu", "salu", "lds", "vmem", "smem", "branch", "s_ctrl"):
        out[k + "_per_launch"] = out[k] / L
    out["valu_mix"] = {op: v / n_valu for op, v in sorted(valu.items(), key=lambda x: -x[1])}
    if args.costs:
        costs = json.load(open(args.costs))
        # cycles per wave64 instruction on one SIMD at the kernel's waves/SIMD
        # (and at one wave alone): unknown opcodes take the default class
        w = str(args.waves)
        cy = 0.0
        cy1 = 0.0
        unknown = collections.Counter()
        for op, v in valu.items():
            c = costs["valu"].get(op)
            if c is None:
                c = costs["valu_default"]
                unknown[op] += v
            cy += v * c[w]
            cy1 += v * c["1"]
        out["valu_simd_cycles_predicted"] = cy / L
        out["valu_wave_cycles_one_wave"] = cy1 / L
        out["valu_unpriced_frac"] = sum(unknown.values()) / n_valu
        out["valu_unpriced_top"] = dict(unknown.most_common(12))
    if args.pmc:
        p = json.load(open(args.pmc))
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if k in p:
                out[k + "_measured"] = p[k]
    hot.sort(reverse=True)
    out["hot_blocks"] = [{"block": k, "executions": e, "instr": n, "valu_share": v / max(1, n_valu)}
                         for v, k, e, n in hot[:25]]
    s = json.dumps(out, indent=1)
    if args.json:
        open(args.json, "w").write(s)
    print(s)


LOC = re.compile(r"^\s*\.loc\s+\d+\s+\d+\s+\d+.*;\s*(\S+):(\d+):\d+")


def lines_cmd(args):
    lines = open(args.inp).read().split("\n")
    start, end = find_kernel(lines, args.kernel)
    blocks = split_blocks(lines, start, end)
    if args.orig:
        _, ob = load_blocks(args.orig, args.kernel)
        sig = lambda bl: [[op for _, op, _ in ins] for _, ins in bl]
        if sig(ob) != sig(blocks):
            raise SystemExit("the -g assembly's blocks differ from the counted build's")
    counts = json.load(open(args.counts))["wave_executions"]
    costs = json.load(open(args.costs))
    w = str(args.waves)
    # the source location in force at each instruction line
    loc, where = "?", {}
    for i in range(start, end):
        m = LOC.match(lines[i])
        if m:
            loc = m.group(1).split("/")[-1] + ":" + m.group(2)
        where[i] = loc
    agg = collections.defaultdict(lambda: [0.0, 0, 0, 0])  # cycles, valu, single-issue, salu
    total = 0.0
    for k, (_, ins) in enumerate(blocks):
        e = counts[k] if k < len(counts) else 0
        if not e:
            continue
        for i, op, t in ins:
            cl = classify(op, t)
            a = agg[where[i]]
            if cl.startswith("valu:"):
                c = costs["valu"].get(op, costs["valu_default"])[w]
                a[0] += e * c
                a[1] += e
                a[2] += e if c > 3.0 else 0
                total += e * c
            elif cl == "salu":
                a[3] += e
    L = max(1, json.load(open(args.counts)).get("launches", 1))
    rows = sorted(agg.items(), key=lambda x: -x[1][0])
    out = [{"loc": k, "cycle_share": round(v[0] / total, 4), "valu_per_launch": v[1] // L,
            "single_issue_frac": round(v[2] / max(1, v[1]), 3), "salu_per_launch": v[3] // L}
           for k, v in rows if v[0] > 0]
    if args.json:
        json.dump({"kernel": kernel_name(lines, start), "rows": out}, open(args.json, "w"), indent=1)
    acc = 0.0
    for r in out[:args.top]:
        acc += r["cycle_share"]
        print(f"{r['loc']:28s} {100 * r['cycle_share']:6.2f} %  cum {100 * acc:6.2f} %  valu/launch "
              f"{r['valu_per_launch']:>12,}  single {r['single_issue_frac']:.2f}")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("instrument")
    a.add_argument("inp")
    a.add_argument("out")
    a.add_argument("--kernel", required=True)
    a.add_argument("--sym", required=True)
    b = sub.add_parser("blocks")
    b.add_argument("inp")
    b.add_argument("--kernel", required=True)
    b.add_argument("--json")
    m = sub.add_parser("model")
    m.add_argument("inp")
    m.add_argument("--kernel", required=True)
    m.add_argument("--counts", required=True)
    m.add_argument("--costs")
    m.add_argument("--waves", type=int, default=4)
    m.add_argument("--pmc")
    m.add_argument("--json")
    ln = sub.add_parser("lines")
    ln.add_argument("inp")
    ln.add_argument("--kernel", required=True)
    ln.add_argument("--counts", required=True)
    ln.add_argument("--costs", required=True)
    ln.add_argument("--orig")
    ln.add_argument("--waves", type=int, default=4)
    ln.add_argument("--top", type=int, default=60)
    ln.add_argument("--json")
    a = ap.parse_args()
    {"instrument": instrument, "blocks": blocks_cmd, "model": model_cmd, "lines": lines_cmd}[a.cmd](a)


if __name__ == "__main__":
    main()
