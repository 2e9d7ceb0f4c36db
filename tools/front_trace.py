"""k_front's timeline (A/B build, round 6): for every block (up to 2,048), the
microseconds from the kernel's first block entry to each phase boundary of
its first item -- ply 1 made, ply 2 counted, ply 2 enumerated, ply-3 counts,
ply-3 scan, the item's ply-3 nodes selected, its ply-4 moves enumerated (depth
7), its offsets found by the look-back, its boards and words stored (wall
clock read by thread 0 after each barrier).  Printed: the median over blocks
of each stamp, and percentiles of entry and done times over all blocks, by
block-index quartile.
GPU tool: DCHESS_LIB=.../libdchess_ab.so python tools/front_trace.py [depth] [shards]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

NB, NW = 2048, 16
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 7
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # shard 0 of N (one rank's work at N GPUs)
eng = dchess.Engine(0)
lib = ctypes.CDLL(os.environ["DCHESS_LIB"])
lib.dc_ab_front_trace.argtypes = [ctypes.c_void_p]
buf = np.zeros(NB * NW, np.uint64)
names = ["ply1", "ply2_count", "ply2_enum", "ply3_count", "ply3_scan", "select", "ply4_enum", "lookback",
         "item_done", "boards_stored", "window0_walked"]
runs = []
for _ in range(6):
    buf[:] = 0
    assert lib.dc_ab_front_trace(buf.ctypes.data) == 0  # (clears nothing: read the previous run's, then rerun)
    if shards > 1:
        eng.perft_shard(dchess.startpos(), depth, 3, 0, shards)
    else:
        eng.perft(dchess.startpos(), depth)
    assert lib.dc_ab_front_trace(buf.ctypes.data) == 0
    t = buf.astype(np.int64).reshape(NB, NW)
    used = t[:, 0] > 0
    t = t[used]
    t0 = t[:, 0].min()
    rel = lambda k: (t[:, k] - t0) / 100.0  # noqa: E731
    q = np.array_split(np.arange(len(t)), 4)
    runs.append({"blocks": int(used.sum()),
                 **{n: float(np.median((t[:, k + 1] - t[:, 0]) / 100.0)) for k, n in enumerate(names)},
                 "entry_p50": float(np.median(rel(0))), "entry_max": float(rel(0).max()),
                 "done_p50": float(np.median(rel(9))), "done_p90": float(np.percentile(rel(9), 90)),
                 "done_max": float(rel(9).max()),
                 **{f"done_med_q{i}": float(np.median(rel(9)[ix])) for i, ix in enumerate(q)},
                 **{f"lookback_med_q{i}": float(np.median(((t[:, 8] - t[:, 0]) / 100.0)[ix])) for i, ix in enumerate(q)},
                 "words_med": float(np.median(t[:, 13])), "boards_med": float(np.median(t[:, 14])),
                 "publish_p50": float(np.median(rel(12))), "publish_p90": float(np.percentile(rel(12), 90)),
                 "publish_max": float(rel(12).max())})
    pub = rel(12)
    slow = np.argsort(-pub)[:8]
    runs[-1]["slowest"] = [[int(np.nonzero(used)[0][i]), round(float(pub[i]), 1), int(t[i, 14]), int(t[i, 13]),
                            round(float((t[i, 6] - t0) / 100.0), 1), round(float((t[i, 5] - t0) / 100.0), 1)]
                           for i in slow]
out = {k: round(float(np.median([r[k] for r in runs[1:]])), 2) for k in runs[0] if k != "slowest"}
out["slowest_last_run(block,publish,boards,words,select,scan)"] = runs[-1]["slowest"]
print(json.dumps({"depth": depth, "shards": shards, "stamps_us": out}))
