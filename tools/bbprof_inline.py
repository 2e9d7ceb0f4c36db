#!/usr/bin/env python3
"""Inclusive per-function (inlined call chain) attribution of a kernel's
basic-block profile (tools/bbprof.py).  Measurement tooling only.

  python tools/bbprof_inline.py CODE_OBJECT.co ASM_G.s --kernel SUBSTR \
      --counts COUNTS.json --costs COSTS.json [--depth N] [--json OUT]

CODE_OBJECT.co and ASM_G.s come from one device compile of the product source
with -gline-tables-only (blocks identical to the counted build: bbprof.py
lines --orig checks that).  Every instruction of the kernel in the code object
is symbolized with llvm-symbolizer --inlines; its dynamic VALU issue cycles
(executions of its block x the opcode's measured cost) are added to every
frame of its inlined chain.  Prints the frames by inclusive share, and the
chain prefixes (caller line -> callee) up to --depth."""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bbprof  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_instrs(dis_lines, name):
    """[(addr, opcode)] of the kernel `name` in llvm-objdump -d output."""
    out, inside = [], False
    for ln in dis_lines:
        if ln.endswith(">:"):
            inside = ("<" + name + ">:") in ln
            continue
        if not inside:
            continue
        m = re.match(r"\s+([a-z_][a-z0-9_]*)\b.*//\s*([0-9A-F]{12}):", ln)
        if m:
            out.append((int(m.group(2), 16), m.group(1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("co")
    ap.add_argument("asm")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--counts", required=True)
    ap.add_argument("--costs", required=True)
    ap.add_argument("--waves", type=int, default=4)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--json")
    a = ap.parse_args()
    lines = open(a.asm).read().split("\n")
    start, end = bbprof.find_kernel(lines, a.kernel)
    name = bbprof.kernel_name(lines, start)
    blocks = bbprof.split_blocks(lines, start, end)
    seq = []  # (block, opcode) in program order
    for k, (_, ins) in enumerate(blocks):
        for _, op, _ in ins:
            seq.append((k, op))
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", a.co], capture_output=True,
                         text=True, check=True).stdout.split("\n")
    ki = kernel_instrs(dis, name)
    if len(ki) != len(seq) or any(op != o2 for (_, op), (_, o2) in zip(ki, seq)):
        # the assembler may print an alias for a few opcodes: compare counts only
        bad = sum(1 for (_, op), (_, o2) in zip(ki, seq) if op != o2)
        if len(ki) != len(seq) or bad > len(seq) // 100:
            raise SystemExit(f"code object and assembly disagree: {len(ki)} vs {len(seq)} instructions, {bad} opcodes")
    sym = subprocess.run([LLVM + "/llvm-symbolizer", "--inlines", "--obj=" + a.co, "--functions=short"],
                         input="\n".join(hex(x) for x, _ in ki) + "\n", capture_output=True, text=True,
                         check=True).stdout
    chains = []
    for rec in sym.strip("\n").split("\n\n"):
        fr = rec.strip("\n").split("\n")
        # pairs (function, file:line:col), innermost first
        chain = []
        for i in range(0, len(fr) - 1, 2):
            fn, loc = fr[i], fr[i + 1]
            loc = loc.split("/")[-1]
            chain.append((fn, ":".join(loc.split(":")[:2])))
        chains.append(chain[::-1])  # outermost first
    if len(chains) != len(ki):
        raise SystemExit(f"symbolizer returned {len(chains)} records for {len(ki)} addresses")
    counts = json.load(open(a.counts))["wave_executions"]
    costs = json.load(open(a.costs))
    w = str(a.waves)
    incl = collections.Counter()
    prefix = collections.Counter()
    total = 0.0
    for (k, op), chain in zip(seq, chains):
        e = counts[k] if k < len(counts) else 0
        if not e or not op.startswith("v_"):
            continue
        c = e * costs["valu"].get(op, costs["valu_default"])[w]
        total += c
        seen = set()
        for fn, _ in chain:
            if fn not in seen:
                incl[fn] += c
                seen.add(fn)
        # call-site prefixes: "f1@line > f2@line > ..." (the line is where the
        # frame calls its callee, i.e. the next frame's call site)
        p = []
        for j, (fn, loc) in enumerate(chain[:a.depth]):
            p.append(f"{fn}@{loc}")
            prefix[" > ".join(p)] += c
    rows = [{"frame": f, "share": round(v / total, 4)} for f, v in incl.most_common()]
    pre = [{"chain": f, "share": round(v / total, 4)} for f, v in prefix.most_common()]
    if a.json:
        json.dump({"kernel": name, "frames": rows, "chains": pre}, open(a.json, "w"), indent=1)
    print("inclusive VALU issue cycles by inlined frame:")
    for r in rows[:a.top]:
        print(f"  {100 * r['share']:6.2f} %  {r['frame']}")
    print(f"call-site chains (depth <= {a.depth}):")
    for r in pre[:a.top]:
        print(f"  {100 * r['share']:6.2f} %  {r['chain']}")


if __name__ == "__main__":
    main()
