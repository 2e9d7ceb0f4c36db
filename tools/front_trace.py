"""k_front's timeline (A/B build, round 6): for the first 64 blocks, the
microseconds from kernel entry to each phase boundary -- ply 1 made, ply 2
counted, ply 2 enumerated, ply-3 counts, ply-3 scan, the first item's ply-3
nodes selected, its ply-4 moves enumerated (depth 7), its offsets found by
the look-back, its boards and words stored (wall clock read by thread 0 after
each barrier).
GPU tool: DCHESS_LIB=.../libdchess_ab.so python tools/front_trace.py [depth]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 7
eng = dchess.Engine(0)
lib = ctypes.CDLL(os.environ["DCHESS_LIB"])
lib.dc_ab_front_trace.argtypes = [ctypes.c_void_p]
buf = np.zeros(64 * 16, np.uint64)
names = ["ply1", "ply2_count", "ply2_enum", "ply3_count", "ply3_scan", "select", "ply4_enum", "lookback",
         "item0_done"]
runs = []
for _ in range(6):
    eng.perft(dchess.startpos(), depth)
    assert lib.dc_ab_front_trace(buf.ctypes.data) == 0
    t = buf.astype(np.int64).reshape(64, 16)
    t0 = t[:, 0].min()
    runs.append({"entry_spread_us": float((t[:, 0].max() - t0) / 100.0),
                 **{n: float(np.median((t[:, k + 1] - t[:, 0]) / 100.0)) for k, n in enumerate(names)},
                 "item0_done_max_us": float((t[:, 9].max() - t0) / 100.0)})
out = {k: round(float(np.median([r[k] for r in runs[1:]])), 2) for k in runs[0]}
print(json.dumps({"depth": depth, "stamps_us_from_entry_median_over_blocks": out}))
