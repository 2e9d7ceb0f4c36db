"""Edit one kernel's device assembly in place (DESIGN.md §3.6 fault study).
  python tools/diag/asm_edit.py FILE.s [KERNEL_SUBSTR] [rule ...]
rules (applied inside the kernel only; instruction index = count of
instruction lines from the kernel's first line):
  none                      identity (checks the pipeline)
  nop_after_asm:N           s_nop N after every inline-asm block
  nop_before_asm:N          s_nop N before every inline-asm block
  nop_after_exec:N          s_nop N after every SALU write of EXEC
  nop_after_vcmp:N          s_nop N after every VOPC / v_cmp writing VCC or SGPRs
  nop_after_sdst:N          s_nop N after every VALU instruction that writes an SGPR or VCC
  nop_before_exec:N         s_nop N before every SALU write of EXEC
  nop_before_salu:N         s_nop N before every SALU instruction (not s_nop / s_waitcnt / branches)
  nop_after_op:OPC:N        s_nop N after every instruction whose opcode starts with OPC
  nop_before_op:OPC:N       s_nop N before every instruction whose opcode starts with OPC
  range:A:B                 restrict the following rules to instruction indices [A, B)
  setprio:N                 s_setprio N before the kernel's first instruction
  split_movb64:0            v_mov_b64_e32 v[a:b], X -> two v_mov_b32 (X = 0, -1 or a register pair)
  vcc_refresh:0             s_mov_b64 vcc, vcc before every s_cbranch_vccz / s_cbranch_vccnz
  vccz_nop:N                s_nop N before every s_cbranch_vccz / s_cbranch_vccnz
  insert_after:IDX:TEXT     insert TEXT after instruction IDX ('~' for a space, '^' for a comma)
  prio_blocks:A:B           wave priority 3 inside instruction indices [A, B), 0 elsewhere: an
                            s_setprio at every branch-target label and at A and B
Prints how many lines were inserted."""
import re
import sys

path = sys.argv[1]
args = sys.argv[2:]
kern = "_ZN2dc9k_count2bINS_9FideRulesELi1EE"
if args and not re.match(r"^(none|nop_|range|setprio|split_|prio_|vcc|insert_)", args[0]):
    kern, args = args[0], args[1:]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(kern) and l.rstrip().endswith(":") or
             (l.startswith(kern) and ": " in l and "@" in l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
INST = re.compile(r"^\s+([a-z_][a-z0-9_]*)\b")
exec_w = re.compile(r"^\s+s_\w+\s+exec\b|^\s+s_\w*saveexec\w*\s")
vcmp = re.compile(r"^\s+v_cmpx?_\w+")
sdst = re.compile(r"^\s+(v_cmpx?_\w+_e32\b|v_(add|sub|subrev)_co_u32_e32\b|v_addc_co_u32_e32\b|v_subb_co_u32_e32\b|"
                  r"v_\w+\s+(vcc|s\[|s\d|exec)|"
                  r"(v_(add|sub|subrev|addc|subb)_co_u32_e64|v_mad_[ui]64_[ui]32|v_div_scale\w*)\s+v[\[\d][^,]*,\s*(vcc|s\[|s\d))")
salu = re.compile(r"^\s+s_(?!nop|waitcnt|cbranch|branch|endpgm|barrier|sleep|setprio)\w+")
out = lines[:start]
idx = 0
lo, hi = 0, 1 << 30
inserted = 0
rules = []
for a in args:
    if a.startswith("range:"):
        _, x, y = a.split(":")
        lo, hi = int(x), int(y)
    elif a.startswith("prio_blocks:"):
        _, x, y = a.split(":")
        rules.append(("prio_blocks:0", int(x), int(y)))
    elif a.startswith("insert_after:"):
        rules.append((a, 0, 1 << 30))
    elif a != "none":
        rules.append((a, lo, hi))
in_asm = False
for i in range(start, end + 1):
    l = lines[i]
    m = INST.match(l)
    is_inst = bool(m) and not l.strip().startswith(";")
    pre, post = [], []
    for r, a0, a1 in rules:
        if r.startswith("prio_blocks"):
            is_label = bool(re.match(r"^\.LBB\d+_\d+:", l))
            if is_label:
                post.append(f"\ts_setprio {3 if a0 <= idx < a1 else 0}")
            elif is_inst and idx in (a0, a1):
                pre.append(f"\ts_setprio {3 if idx == a0 else 0}")
            continue
        if not (a0 <= idx < a1):
            continue
        kind = r.split(":")
        n = int(kind[-1]) if kind[-1].lstrip("-").isdigit() else 0
        if kind[0] == "nop_after_asm" and ";;#ASMEND" in l:
            post.append(f"\ts_nop {n}")
        elif kind[0] == "nop_before_asm" and ";;#ASMSTART" in l:
            pre.append(f"\ts_nop {n}")
        elif kind[0] == "nop_after_exec" and is_inst and exec_w.match(l):
            post.append(f"\ts_nop {n}")
        elif kind[0] == "nop_after_vcmp" and is_inst and vcmp.match(l):
            post.append(f"\ts_nop {n}")
        elif kind[0] == "nop_after_sdst" and is_inst and sdst.match(l):
            post.append(f"\ts_nop {n}")
        elif kind[0] == "setprio" and is_inst and idx == 0:
            pre.append(f"\ts_setprio {n}")
        elif kind[0] == "vcc_refresh" and is_inst and m.group(1) in ("s_cbranch_vccz", "s_cbranch_vccnz"):
            pre.append("\ts_mov_b64 vcc, vcc")
        elif r.startswith("insert_after:") and is_inst and idx == int(r.split(":")[1]):
            post.append("\t" + r.split(":", 2)[2].replace("~", " ").replace("^", ","))
        elif kind[0] == "vccz_nop" and is_inst and m.group(1) in ("s_cbranch_vccz", "s_cbranch_vccnz"):
            pre.append(f"\ts_nop {n}")
        elif kind[0] == "nop_before_exec" and is_inst and exec_w.match(l):
            pre.append(f"\ts_nop {n}")
        elif kind[0] == "nop_before_salu" and is_inst and salu.match(l):
            pre.append(f"\ts_nop {n}")
        elif kind[0] == "nop_after_op" and is_inst and m.group(1).startswith(kind[1]):
            post.append(f"\ts_nop {n}")
        elif kind[0] == "nop_before_op" and is_inst and m.group(1).startswith(kind[1]):
            pre.append(f"\ts_nop {n}")
    for r, a0, a1 in rules:
        if r.startswith("split_movb64") and a0 <= idx < a1 and is_inst:
            mm = re.match(r"^(\s+)v_mov_b64_e32\s+v\[(\d+):(\d+)\],\s*(\S+)\s*$", l)
            if mm:
                ind, a, b, x = mm.group(1), mm.group(2), mm.group(3), mm.group(4)
                ms = re.match(r"v\[(\d+):(\d+)\]", x)
                if ms:
                    lo_src, hi_src = "v" + ms.group(1), "v" + ms.group(2)
                elif x in ("0", "-1"):
                    lo_src = hi_src = x
                else:
                    continue
                l = f"{ind}v_mov_b32_e32 v{a}, {lo_src}\n{ind}v_mov_b32_e32 v{b}, {hi_src}"
                inserted += 1
    out += pre + [l] + post
    inserted += len(pre) + len(post)
    if is_inst:
        idx += 1
out += lines[end + 1:]
open(path, "w").write("\n".join(out))
print(f"asm_edit: kernel {kern} lines {start}-{end}, {idx} instructions, {inserted} lines inserted", file=sys.stderr)
