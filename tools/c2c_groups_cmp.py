"""Compares the per-group leaf counts dumped by tools/c2c_groups.py
(gpurun_out/groups_<TAG>_d<d>_r<run>.npy) between builds and runs:
per group, the leaves it added to each root tag (a block's cumulative
histogram differenced in clock order).  Prints the groups whose counts differ
from the reference build's first run.
usage: python tools/c2c_groups_cmp.py <ref_tag> <tag> <depth> <n_groups>"""
import glob
import sys
import numpy as np


def per_group(path, n_groups):
    rec = np.load(path)[:n_groups]
    hist, blk, clk = rec[:, :256].astype(np.int64), rec[:, 256], rec[:, 257]
    out = np.zeros_like(hist)
    for b in np.unique(blk):
        rows = np.where(blk == b)[0]
        rows = rows[np.argsort(clk[rows])]
        prev = np.zeros(256, np.int64)
        for r in rows:
            out[r] = hist[r] - prev
            prev = hist[r]
    return out, blk


if __name__ == "__main__":
    ref_tag, tag, d, n = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    ref, _ = per_group(f"gpurun_out/groups_{ref_tag}_d{d}_r0.npy", n)
    for p in sorted(glob.glob(f"gpurun_out/groups_{tag}_d{d}_r*.npy")):
        g, blk = per_group(p, n)
        diff = (g - ref).sum(axis=1)
        bad = np.nonzero(diff)[0]
        print(p, "groups differing:", len(bad), "sum of deltas", int(diff.sum()))
        for i in bad[:60]:
            print(f"   group {i} block {int(blk[i])} delta {int(diff[i])} ref {int(ref[i].sum())}")
