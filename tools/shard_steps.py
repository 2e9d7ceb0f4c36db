"""Per-rank perft step of an N-rank run, measured on ONE GPU: for every shard r
of N, the bench's timed path (dc_perft_repeat_device, K runs back to back, no
host round trip) is timed on its own, and the kernel breakdown of one shard is
taken with HIP events.  The slowest shard bounds the N-GPU step (the exchange
step -- one bucketed all-reduce per K steps -- is not included).  Prints one
JSON line per N with the projected leaves/s and strong-scaling efficiency.
GPU tool; the totals are checked against the golden count."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 7
split = int(os.environ.get("SPLIT", "3"))
K = int(os.environ.get("RUNS", "20"))
WANT = {6: 120909581, 7: 3282734510}.get(depth)
e = dchess.Engine(0)
s = dchess.startpos()
e.perft(s, depth)
W = 258
base = None
for N in [int(x) for x in os.environ.get("RANKS", "1 2 4 8").split()]:
    ms, tot = [], 0
    for r in range(N):
        buf = e.alloc(K * W * 8)
        e.perft_repeat_device(s, depth, split, r, N, 1, buf)  # capture outside the timing
        e.synchronize()
        t0 = time.perf_counter()
        e.perft_repeat_device(s, depth, split, r, N, K, buf)
        e.synchronize()
        ms.append((time.perf_counter() - t0) / K * 1e3)
        res = buf.download(np.uint64, K * W).reshape(K, W)
        buf.free()
        tot += int(res[0, 257])
    e.reset_stats()
    e.set_profiling(True)
    e.perft_shard(s, depth, split, 0, N)
    e.set_profiling(False)
    ks = {k: round(e.kernel_stats(k)["total_ms"], 4) for k in ("expand_top", "expand_count", "scan", "expand_write",
                                                               "count2")}
    step = max(ms)
    base = base or step
    print(json.dumps({"depth": depth, "split": split, "ranks": N, "total_ok": WANT is None or tot == WANT,
                      "rank_ms": [round(x, 4) for x in ms], "step_ms": round(step, 4),
                      "projected_leaves_per_s": (WANT or tot) / (step / 1e3),
                      "strong_scaling_eff": round(base / (N * step), 3), "shard0_kernels_ms": ks}), flush=True)
