"""Summary of a rocprofv3 --kernel-trace database (rocpd .db): per-kernel
median / min duration, and for the perft repeat sequence (k_front or the
legacy chain, then k_count3c, then k_copy_result) the median span of one run
from its first kernel's start to the copy's end and the gaps between kernels.
usage: python tools/trace_summary.py DIR_OR_DB [...]"""
import collections
import glob
import os
import sqlite3
import sys


def load(path):
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = []
    for db in dbs:
        con = sqlite3.connect(db)
        rows += list(con.execute("select name, start, end from kernels order by start"))
    rows.sort(key=lambda r: r[1])
    return [(n.split("(")[0].replace("void ", ""), s, e) for n, s, e in rows]


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


for path in sys.argv[1:]:
    seq = load(path)
    per = collections.defaultdict(list)
    for n, s, e in seq:
        per[n].append((e - s) / 1e3)
    print(path)
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:58]:58s} n={len(v):5d} med={med(v):9.2f} us  min={min(v):9.2f}")
    # runs: from the kernel after a k_copy_result to the next k_copy_result's end
    spans, gaps = [], []
    start = None
    for i, (n, s, e) in enumerate(seq):
        if start is None:
            start = s
        if i:
            gaps.append((s - seq[i - 1][2]) / 1e3)
        if "k_copy_result" in n:
            spans.append((e - start) / 1e3)
            start = None
    if spans:
        print(f"  run span (first kernel start .. copy end): med {med(spans):.2f} us over {len(spans)} runs;"
              f" kernel-to-kernel gap med {med(gaps):.2f} us")
