"""perft(7) steps on one context against the same steps split over 2-4 contexts
(streams) run concurrently: does one run's front end hide behind another's
final stage?  (Round 4 measured a strict alternation over two contexts at
1.03 vs 0.53 ms per step; this enqueues each context's whole share at once.)
  python tools/overlap_perft.py [--steps 32] [--depth 7] [--ctx 2]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=32)
ap.add_argument("--depth", type=int, default=7)
ap.add_argument("--ctx", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--torch", action="store_true", help="initialise torch's HIP runtime first (as bench.py does)")
ap.add_argument("--shards", type=int, default=1, help="time shard 0 of N (one rank's work at N GPUs)")
a = ap.parse_args()
if a.torch:
    import torch
    assert torch.cuda.is_available()
    torch.cuda.synchronize()
W = 258
WANT = {6: 120909581, 7: 3282734510, 8: 88792516787}  # REF
pos = dchess.startpos()
engs = [dchess.Engine(0) for _ in range(a.ctx)]
bufs = [e.alloc(a.steps * W * 8) for e in engs]
for e, b in zip(engs, bufs):
    for k in (1, 8, a.steps // a.ctx):
        e.perft_repeat_device(pos, a.depth, 3, 0, a.shards, k, b)
    e.synchronize()


def check(b, n):
    r = b.download(np.uint64, n * W).reshape(n, W)
    if a.shards == 1:
        assert (r[:, 257] == WANT[a.depth]).all(), r[:, 257][:4]
    else:  # one shard: every run the same count
        assert (r[:, 257] == r[0, 257]).all() and r[0, 257] > 0, r[:, 257][:4]


out = {"depth": a.depth, "steps": a.steps, "ctx": a.ctx, "torch": a.torch, "shards": a.shards, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
for rep in range(a.reps):
    t0 = time.perf_counter()
    engs[0].perft_repeat_device(pos, a.depth, 3, 0, a.shards, a.steps, bufs[0])
    engs[0].synchronize()
    one = time.perf_counter() - t0
    check(bufs[0], a.steps)
    share = a.steps // a.ctx
    t0 = time.perf_counter()
    for i, (e, b) in enumerate(zip(engs, bufs)):
        e.perft_repeat_device(pos, a.depth, 3, 0, a.shards, share, b)
    for e in engs:
        e.synchronize()
    many = time.perf_counter() - t0
    for b in bufs:
        check(b, share)
    out.setdefault("one_ctx_ms_per_step", []).append(round(1e3 * one / a.steps, 4))
    out.setdefault("split_ms_per_step", []).append(round(1e3 * many / (share * a.ctx), 4))
print(json.dumps(out))
