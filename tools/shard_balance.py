"""Per-shard time and leaves of perft(startpos, D) split S over R shards on one
GPU: the imbalance a contiguous-range sharding leaves for --gpus R."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 7
e = dchess.Engine(0)
s = dchess.startpos()
e.perft(s, depth)  # first touch of the level buffers (16 GB speculative caps) outside the timings
for split in [int(x) for x in os.environ.get("SPLITS", "3 4").split()]:
    for R in (2, 4, 8):
        rows = []
        for r in range(R):
            e.perft_shard(s, depth, split, r, R)
            t0 = time.perf_counter()
            for _ in range(3):
                tot, _, _ = e.perft_shard(s, depth, split, r, R)
            rows.append((tot, (time.perf_counter() - t0) / 3 * 1e3))
        ms = [x[1] for x in rows]
        print(json.dumps({"depth": depth, "split": split, "shards": R, "leaves": [x[0] for x in rows],
                          "ms": [round(x, 3) for x in ms], "max_over_mean": max(ms) / (sum(ms) / R)}), flush=True)
