"""Victim perft runs beside co-resident noise waves (DESIGN.md §3.6 study).

DCHESS_LIB=<victim build> [DC_DIAG_GRID=96] python tools/diag/noise_check.py \
    --rules fide|ref --depth D --kinds -1,0,1,2,3,4,5 [--blocks 512] [names...]
kind -1 = no noise.  Prints one JSON line per kind: the perft differences
against the golden (FIDE: published counts; REF: startpos goldens)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="*", default=["kiwipete", "pos5", "pos6"])
ap.add_argument("--rules", default="fide")
ap.add_argument("--depth", type=int, default=5)
ap.add_argument("--kinds", default="-1,0,1,2,3,4,5")
ap.add_argument("--blocks", type=int, default=512)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ms", type=float, default=0)
args = ap.parse_args()
N = C.CDLL(os.path.join(REPO, "tools", "diag", "libnoise.so"))
N.noise_start.argtypes = [C.c_int, C.c_int, C.c_double]
og = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_golden.json")))
eng = dchess.Engine(0)
fide = args.rules == "fide"


def want(name):
    if fide:
        return og["perft_fide"][name]["perft"][str(args.depth)]
    return og["perft_ref"]["startpos"][str(args.depth)]["total"]


def pos(name):
    return dchess.pos_from_fen(og["perft_fide"][name]["fen"]) if fide else dchess.startpos()


rules = dchess.RULES_FIDE if fide else dchess.RULES_REF
names = args.names if fide else ["startpos"]
for n in names:  # warm up: graphs captured, buffers sized, outside the noise
    eng.perft(pos(n), args.depth, rules=rules)
for kind in [int(k) for k in args.kinds.split(",")]:
    out = {}
    t0 = time.time()
    budget = args.ms or 400.0 * args.reps * len(names) * (1 if args.depth <= 5 else 4)
    if kind >= 0:
        assert N.noise_start(kind, args.blocks, budget) == 0
        time.sleep(0.05)
    for n in names:
        for _ in range(args.reps):
            t, _, _ = eng.perft(pos(n), args.depth, rules=rules)
            out.setdefault(n, []).append(int(t) - want(n))
    elapsed = time.time() - t0
    if kind >= 0:
        assert N.noise_wait() == 0
    print(json.dumps({"lib": os.environ.get("DCHESS_LIB", "product"), "grid": os.environ.get("DC_DIAG_GRID"),
                      "rules": args.rules, "depth": args.depth, "noise_kind": kind, "noise_ms": budget if kind >= 0 else 0,
                      "victim_s": round(elapsed, 3), "diffs": out}), flush=True)
