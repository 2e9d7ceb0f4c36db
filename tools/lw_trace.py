"""k_level_write<MW>'s per-block timeline (A/B build): for the move-word level of
perft(7) (ply 5 written as 4-byte words from ply 4), the spread of block entry
and exit times and the median block's phases (scan, enumeration, writes), in
microseconds from the first block's entry.
GPU tool: DCHESS_LIB=.../libdchess_ab.so python tools/lw_trace.py"""
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
lib.dc_ab_lw_trace.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 4, np.uint64)
out = []
for _ in range(3):
    buf[:] = 0
    eng.perft(dchess.startpos(), int(os.environ.get("DEPTH", "7")))
    assert lib.dc_ab_lw_trace(buf.ctypes.data) == 0
    t = buf.astype(np.int64).reshape(-1, 4)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    busy = t[t[:, 3] > t[:, 1]]  # blocks that had a chunk
    q = lambda x: [round(float(np.percentile(x, p)) / 100.0, 2) for p in (0, 50, 100)]
    out.append({"blocks": int(len(t)), "busy_blocks": int(len(busy)),
                "entry_us_min_med_max": q(t[:, 0] - t0), "exit_us_min_med_max": q(t[:, 3] - t0),
                "scan_us_med": round(float(np.median(busy[:, 1] - busy[:, 0])) / 100.0, 2),
                "enumerate_us_med": round(float(np.median(busy[:, 2] - busy[:, 1])) / 100.0, 2),
                "write_us_med": round(float(np.median(busy[:, 3] - busy[:, 2])) / 100.0, 2)})
print(json.dumps(out[-1]))
