"""FIDE suite at depth 5 (BASELINE configs[2]) timed two ways on one GPU:
sequential (one context, one position after another, as bench.py's
fide_suite_d5 leg) and concurrent (one context -- one stream -- per position,
all six positions' repeat runs enqueued before any is waited for).
  python tools/suite_time.py [--steps 16] [--split 3]"""
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
ap.add_argument("--steps", type=int, default=16)
ap.add_argument("--split", type=int, default=3)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
og = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_golden.json")))["perft_fide"]
names = ["kiwipete", "pos3", "pos4", "pos5", "pos6", "startpos"]
F = dchess.RULES_FIDE
W = 258
pos = {n: dchess.pos_from_fen(og[n]["fen"]) for n in names}
want = {n: og[n]["perft"]["5"] for n in names}
engs = {n: dchess.Engine(0) for n in names}
bufs = {n: engs[n].alloc(args.steps * W * 8) for n in names}
for n in names:  # captures (plain run, one-run graph and the batch graph)
    for k in (1, 8):
        engs[n].perft_repeat_device(pos[n], 5, args.split, 0, 1, k, bufs[n], rules=F)
    engs[n].synchronize()


def check(n):
    res = bufs[n].download(np.uint64, args.steps * W).reshape(args.steps, W)
    assert (res[:, 257] == want[n]).all(), (n, res[:, 257][:3], want[n])


out = {"steps": args.steps}
for rep in range(args.reps):
    t0 = time.perf_counter()
    for n in names:  # sequential: as the bench leg (one position at a time)
        engs[n].perft_repeat_device(pos[n], 5, args.split, 0, 1, args.steps, bufs[n], rules=F)
        engs[n].synchronize()
    seq = time.perf_counter() - t0
    for n in names:
        check(n)
    t0 = time.perf_counter()
    for n in names:  # concurrent: every stream busy before any wait
        engs[n].perft_repeat_device(pos[n], 5, args.split, 0, 1, args.steps, bufs[n], rules=F)
    for n in names:
        engs[n].synchronize()
    conc = time.perf_counter() - t0
    for n in names:
        check(n)
    out.setdefault("seq_ms_per_step", []).append(round(1e3 * seq / args.steps, 4))
    out.setdefault("conc_ms_per_step", []).append(round(1e3 * conc / args.steps, 4))
out["leaves_per_step"] = sum(want.values())
out["grid"] = os.environ.get("DC_DIAG_GRID")
out["lib"] = os.environ.get("DCHESS_LIB", "product")
print(json.dumps(out))
