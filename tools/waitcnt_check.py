"""Independent s_waitcnt checker for a gfx9/CDNA kernel in hipcc's .s output.

Why: round 2's struct-of-arrays build of c2c_group gave timing-dependent wrong
perft counts.  One class of fault that depends on timing
only is a register consumed (or overwritten) while a memory operation that
writes it is still in flight -- a missing or too-weak s_waitcnt.  This tool
re-derives the waits the hardware needs, independently of the compiler's
SIInsertWaitcnts, and reports every instruction that touches a register with
an outstanding load.

Model (CDNA3/4, gfx9 counters):
  * vmcnt: every VMEM op (buffer/global/scratch/flat loads, stores, atomics)
    enters one in-order queue; s_waitcnt vmcnt(N) retires all but the newest N.
  * lgkmcnt: LDS ops retire in order; SMEM (s_load*) may retire out of order,
    so while one is outstanding only lgkmcnt(0) is taken to retire anything.
  * Across the CFG the outstanding queues of all predecessors are merged
    position by position from the newest entry (a forward fixpoint).
Any operand (read or write) that overlaps the destination of an outstanding
load is reported: reading it gets a stale value, writing it races the return.

usage: python tools/waitcnt_check.py file.s [kernel-substring ...]
"""
import re
import sys

REG = re.compile(r"\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b|\b(vcc|exec|m0)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out.update(f"{k}{i}" for i in range(a, b + 1))
        elif m.group(4):
            out.add(f"{m.group(4)}{m.group(5)}")
    return out


def split_ops(rest):
    # operands are comma separated; modifiers (offset:, sc0, dpp controls) follow
    return [o.strip() for o in rest.split(",")]


def classify(mn, ops):
    """-> (counter, dst_regs, all_regs) ; counter in {None,'vm','lds','smem','flat'}"""
    allr = set()
    for o in ops:
        allr |= regs(o)
    first = regs(ops[0]) if ops and ops[0] else set()
    if mn.startswith(("global_", "buffer_", "scratch_")):
        if "load" in mn and " lds" not in " ".join(ops):
            return "vm", first, allr
        if "atomic" in mn and any("sc0" in o or "glc" in o for o in ops):
            return "vm", first, allr
        return "vm", set(), allr
    if mn.startswith("flat_"):
        if "load" in mn or ("atomic" in mn and any("sc0" in o or "glc" in o for o in ops)):
            return "flat", first, allr
        return "flat", set(), allr
    if mn.startswith("ds_"):
        ret = ("read" in mn or "_rtn" in mn or "bpermute" in mn or "permute" in mn or "swizzle" in mn
               or "consume" in mn or "append" in mn)
        return "lds", (first if ret else set()), allr
    if mn.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime")):
        return "smem", first, allr
    return None, set(), allr


def parse(lines):
    """-> list of blocks: (label, [(lineno, mnemonic, ops, raw)], succ_labels, falls_through)"""
    blocks, cur_label, cur = [], "__entry", []
    def close(ft=True, succ=()):
        blocks.append([cur_label, cur, list(succ), ft])
    for ln, raw in lines:
        s = raw.split(";")[0].strip()
        if not s or s.startswith("//"):
            continue
        if s.endswith(":"):
            if cur or cur_label != "__entry" or blocks:
                close()
            cur_label, cur = s[:-1], []
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        ops = split_ops(parts[1]) if len(parts) > 1 else []
        cur.append((ln, mn, ops, raw.rstrip()))
        if mn == "s_branch":
            close(False, [ops[0]])
            cur_label, cur = f"__after{ln}", []
        elif mn.startswith("s_cbranch"):
            close(True, [ops[0]])
            cur_label, cur = f"__after{ln}", []
        elif mn in ("s_endpgm", "s_setpc_b64"):
            close(False)
            cur_label, cur = f"__after{ln}", []
    if cur:
        close()
    return blocks


def merge(a, b):
    """queues are tuples of frozensets, oldest first; align newest entries"""
    n = max(len(a), len(b))
    ra, rb = list(reversed(a)), list(reversed(b))
    out = []
    for i in range(n):
        x = ra[i] if i < len(ra) else frozenset()
        y = rb[i] if i < len(rb) else frozenset()
        out.append(x | y)
    return tuple(reversed(out))


def merge_state(s, t):
    if s is None:
        return t
    return (merge(s[0], t[0]), merge(s[1], t[1]), s[2] | t[2])


VM_MAX, LGKM_MAX = 63, 15
WAIT = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")


def step(state, ins, report):
    vm, lds, smem = list(state[0]), list(state[1]), set(state[2])
    ln, mn, ops, raw = ins
    if mn == "s_waitcnt":
        w = dict((k, int(v)) for k, v in WAIT.findall(" ".join(ops)))
        if "vmcnt" in w:
            n = w["vmcnt"]
            vm = vm[len(vm) - n:] if n < len(vm) else vm
            if n == 0:
                vm = []
        if "lgkmcnt" in w:
            n = w["lgkmcnt"]
            if n == 0:
                lds, smem = [], set()
            elif not smem:
                lds = lds[len(lds) - n:] if n < len(lds) else lds
        return (tuple(vm), tuple(lds), frozenset(smem))
    cnt, dst, allr = classify(mn, ops)
    pending = set()
    for e in vm:
        pending |= e
    for e in lds:
        pending |= e
    pending |= smem
    hit = allr & pending
    if hit and report is not None:
        report.append((ln, raw.strip(), sorted(hit)))
    if cnt == "vm":
        vm.append(frozenset(dst))
    elif cnt == "flat":
        vm.append(frozenset(dst))
        lds.append(frozenset(dst))
    elif cnt == "lds":
        lds.append(frozenset(dst))
    elif cnt == "smem":
        smem |= dst
    # the counters saturate (vmcnt 6 bits, lgkmcnt 4 bits): the hardware stalls
    # issue rather than exceed them, so older entries have retired
    return (tuple(vm[-VM_MAX:]), tuple(lds[-LGKM_MAX:]), frozenset(smem))


def check(lines):
    blocks = parse(lines)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    succs = []
    for i, (lab, ins, succ, ft) in enumerate(blocks):
        s = [idx[x] for x in succ if x in idx]
        if ft and i + 1 < len(blocks):
            s.append(i + 1)
        succs.append(s)
    empty = ((), (), frozenset())
    inn = [None] * len(blocks)
    inn[0] = empty
    work = [0]
    while work:
        i = work.pop()
        st = inn[i]
        for ins in blocks[i][1]:
            st = step(st, ins, None)
        for j in succs[i]:
            new = merge_state(inn[j], st)
            if new != inn[j]:
                inn[j] = new
                work.append(j)
    report = []
    for i, b in enumerate(blocks):
        st = inn[i] if inn[i] is not None else empty
        for ins in b[1]:
            st = step(st, ins, report)
    return report


def kernels(path):
    lines = open(path).read().split("\n")
    out, name, body = {}, None, []
    for i, l in enumerate(lines, 1):
        m = re.match(r"^(_Z\w+):\s*;\s*@", l)
        if m:
            name, body = m.group(1), []
            continue
        if name is not None:
            body.append((i, l))
            if "s_endpgm" in l and not l.strip().startswith(";"):
                # a kernel may have several s_endpgm; keep reading until the next .Lfunc_end
                pass
            if l.startswith(".Lfunc_end"):
                out[name] = body
                name = None
    return out


if __name__ == "__main__":
    path = sys.argv[1]
    subs = sys.argv[2:]
    total = 0
    for name, body in kernels(path).items():
        if subs and not any(s in name for s in subs):
            continue
        rep = check(body)
        total += len(rep)
        print(f"{name}: {len(rep)} operand(s) touching an in-flight load's destination")
        for ln, raw, hit in rep[:40]:
            print(f"   line {ln}: {raw}    <- {','.join(hit)}")
    sys.exit(1 if total else 0)
