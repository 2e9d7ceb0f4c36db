"""Per-block timeline of k_count2c (A/B build, DC_C2C_PHASE=8): for one
perft(startpos, D) launch, when each block started and finished, how many
256-parent chunks it took, how long it waited on the chunk counter, and which
XCD it ran on.  Prints a JSON summary (tail = the last block's exit minus the
median exit; wait share = counter round trips over the block's lifetime).
GPU tool; run via tools/ab_trace.sh."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

assert os.environ.get("DC_C2C_PHASE") == "8", "run with DC_C2C_PHASE=8 and the A/B library"
depth = int(os.environ.get("DEPTH", "7"))
eng = dchess.Engine(0)
pos = dchess.startpos()
tot = None
for _ in range(3):
    tot, _, _ = eng.perft(pos, depth)
lib = ctypes.CDLL(os.environ["DCHESS_LIB"])
lib.dc_ab_c2c_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
W = 8
buf = np.zeros(4096 * W, np.uint64)
assert lib.dc_ab_c2c_trace(buf.ctypes.data, buf.size) == 0
grid = int(buf[6])
r = buf[:grid * W].reshape(grid, W).astype(np.int64)
t0 = r[:, 0].min()
ent, ext, ch, wait, xcc = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0, r[:, 2], r[:, 3] / 100.0, r[:, 4]
life = ext - ent
out = {"depth": depth, "total": tot, "grid": grid, "chunks": int(ch.sum()),
       "entry_us": [round(float(np.percentile(ent, q)), 2) for q in (0, 50, 100)],
       "exit_us": [round(float(np.percentile(ext, q)), 2) for q in (0, 10, 50, 90, 100)],
       "tail_us": round(float(ext.max() - np.median(ext)), 2),
       "chunks_per_block": [int(ch.min()), float(np.median(ch)), int(ch.max())],
       "counter_wait_share": round(float(wait.sum() / life.sum()), 4),
       "counter_wait_us_per_chunk": round(float(wait.sum() / max(ch.sum() + grid, 1)), 3),
       "per_xcc": {int(x): {"blocks": int((xcc == x).sum()), "chunks": int(ch[xcc == x].sum()),
                            "exit_max_us": round(float(ext[xcc == x].max()), 2),
                            "wait_us_per_chunk": round(float(wait[xcc == x].sum() / max(ch[xcc == x].sum(), 1)), 3)}
                   for x in sorted(set(xcc.tolist()))}}
print(json.dumps(out))
