"""k_expand_top's timeline (A/B build): per ply of the top expansion, the
microseconds spent counting, scanning, enumerating into the LDS slots and
making/storing the children (wall clock read by thread 0 after each barrier).
GPU tool: DCHESS_LIB=.../libdchess_ab.so python tools/top_trace.py"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

eng = dchess.Engine(0)
lib = ctypes.CDLL(os.environ["DCHESS_LIB"])
lib.dc_ab_top_trace.argtypes = [ctypes.c_void_p]
buf = np.zeros(20, np.uint64)
rows = []
for _ in range(5):
    eng.perft(dchess.startpos(), int(os.environ.get("DEPTH", "7")))
    assert lib.dc_ab_top_trace(buf.ctypes.data) == 0
    t = buf.astype(np.int64).reshape(4, 5)
    rows.append([[(t[p, k + 1] - t[p, k]) / 100.0 for k in range(4)] for p in (1, 2, 3)])
r = np.median(np.array(rows), axis=0)
print(json.dumps({f"ply{p + 1}": dict(zip(["count", "scan", "enumerate", "make"], [round(float(x), 2) for x in r[p]]))
                  for p in range(3)} | {"total_us": round(float(r.sum()), 2)}))
