"""Reports scratch reloads (scratch_load ... offset:K) that some path from the
kernel entry reaches without a scratch_store to the same bytes: such a reload
returns whatever an earlier wave or kernel left in that private slot, which
depends on wave placement and timing.  Must-stored byte sets, intersected at
CFG merges (forward fixpoint over tools/waitcnt_check.py's block parser).
usage: python tools/scratch_init_check.py file.s [kernel-substring ...]"""
import re
import sys
from waitcnt_check import parse, kernels

OFF = re.compile(r"offset:(-?\d+)")
WIDTH = {"dword": 4, "dwordx2": 8, "dwordx3": 12, "dwordx4": 16, "short": 2, "byte": 1, "ushort": 2, "ubyte": 1,
         "sshort": 2, "sbyte": 1}


def access(mn, ops):
    if not mn.startswith("scratch_"):
        return None
    kind = "store" if "store" in mn else "load"
    w = WIDTH[mn.split("_")[-1]]
    m = OFF.search(" ".join(ops))
    o = int(m.group(1)) if m else 0
    # only the "off, off offset:K" form (a fixed slot) is tracked
    if kind == "store" and not (len(ops) > 2 and ops[0] == "off"):
        return None
    return kind, frozenset(range(o, o + w))


def check(body):
    blocks = parse(body)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    succ = []
    for i, (lab, ins, s, ft) in enumerate(blocks):
        t = [idx[x] for x in s if x in idx]
        if ft and i + 1 < len(blocks):
            t.append(i + 1)
        succ.append(t)
    ALL = None  # top
    inn = [ALL] * len(blocks)
    inn[0] = frozenset()
    seen = [False] * len(blocks)
    work = [0]
    while work:
        i = work.pop()
        st = inn[i]
        seen[i] = True
        for ln, mn, ops, raw in blocks[i][1]:
            a = access(mn, ops)
            if a and a[0] == "store":
                st = st | a[1]
        for j in succ[i]:
            new = st if inn[j] is ALL else (inn[j] & st)
            if new != inn[j] or not seen[j]:
                inn[j] = new
                work.append(j)
    rep = []
    for i, b in enumerate(blocks):
        st = inn[i] if inn[i] is not ALL else frozenset()
        for ln, mn, ops, raw in b[1]:
            a = access(mn, ops)
            if a and a[0] == "load" and not a[1] <= st:
                rep.append((ln, raw.strip(), sorted(a[1] - st)))
            if a and a[0] == "store":
                st = st | a[1]
    return rep


if __name__ == "__main__":
    tot = 0
    for name, body in kernels(sys.argv[1]).items():
        if len(sys.argv) > 2 and not any(s in name for s in sys.argv[2:]):
            continue
        rep = check(body)
        tot += len(rep)
        if rep:
            print(f"{name}: {len(rep)} reload(s) reachable before any store of their bytes")
            for ln, raw, missing in rep[:20]:
                print(f"   line {ln}: {raw}   bytes {missing[0]}..{missing[-1]}")
    print("total", tot)
