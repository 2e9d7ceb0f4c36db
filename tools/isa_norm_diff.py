"""Compare two kernels' instruction streams modulo register numbers and labels
(diagnostics for DESIGN.md §3.6): prints the opcode sequence alignment summary
and the first differing regions.
  python tools/isa_norm_diff.py A.k1.s B.k1.s [context]"""
import difflib
import re
import sys


def norm(path, keep_regs=False):
    out = []
    for ln in open(path):
        s = ln.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        if not keep_regs:
            s = re.sub(r"\bv\[\d+:\d+\]", "V2", s)
            s = re.sub(r"\bs\[\d+:\d+\]", "S2", s)
            s = re.sub(r"\bv\d+\b", "V", s)
            s = re.sub(r"\bs\d+\b", "S", s)
            s = re.sub(r"\.LBB\d+_\d+", "L", s)
        out.append(s)
    return out


def main():
    a, b = norm(sys.argv[1]), norm(sys.argv[2])
    ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    sm = difflib.SequenceMatcher(None, a, b, autojunk=False)
    print(f"{sys.argv[1]}: {len(a)} insts, {sys.argv[2]}: {len(b)} insts, ratio {sm.ratio():.4f}")
    ops = [o for o in sm.get_opcodes() if o[0] != "equal"]
    print(f"{len(ops)} differing regions")
    for tag, i1, i2, j1, j2 in ops[:int(sys.argv[4]) if len(sys.argv) > 4 else 40]:
        print(f"--- {tag} A[{i1}:{i2}] B[{j1}:{j2}]")
        for x in a[max(0, i1 - ctx):i1]:
            print("   ", x)
        for x in a[i1:i2]:
            print(" - ", x)
        for x in b[j1:j2]:
            print(" + ", x)


if __name__ == "__main__":
    main()
