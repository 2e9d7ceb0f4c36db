"""Deep REF perft pins -- TEST INFRASTRUCTURE.

Run:  python tests/golden/make_deep_golden.py [--threads 8] [--max-depth 9]
      (refcpu pins ~10 min on 8 cores; fastcpu perft(8) ~10 min, perft(9) ~2.5 h)

Round 1 pinned REF perft beyond depth 4 only by fastcpu (the mailbox engine),
tied to refcpu -- the literal restatement of /root/reference/core/src/chess.rs
-- by move-set equality.  This script runs refcpu's brute force (every one of
the 4096 (from,to) pairs through validate_move at every interior node, the
reference's own call, chess.rs:82-125) as deep as a few minutes allow and
records, per item, which engines agreed:

  startpos perft(5) divide                    refcpu == fastcpu (4,896,998 leaves)
  startpos perft(6), the subtrees of two root moves   refcpu == fastcpu
  the standard-suite FENs at REF depth 4      refcpu == fastcpu
  24 random REF positions at depth 3          refcpu == fastcpu
  startpos perft(8), perft(9) divide          fastcpu only (refcpu would need
                                              ~1e13 validate_move calls)

Output: tests/golden/ref_deep.json (rewritten after every item).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import oracle_lib as O  # noqa: E402
from make_golden import FIDE_SUITE, random_positions  # noqa: E402


def ref_divide_by_move(rdiv, rm):
    """refcpu's divide (indexed 64*from + to) in fastcpu's root-move order."""
    return [int(rdiv[(int(m) & 63) * 64 + ((int(m) >> 6) & 63)]) for m in rm]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--max-depth", type=int, default=9, help="deepest fastcpu-only startpos perft")
    ap.add_argument("--out", default=os.path.join(HERE, "ref_deep.json"))
    args = ap.parse_args()
    th = args.threads
    out = {}
    if os.path.exists(args.out):
        out = json.load(open(args.out))

    def save():
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)

    start = O.Pos()
    cells0 = O.startpos_cells()
    # ---------------------------------------------------- startpos perft(5) divide
    if "startpos_d5" not in out:
        t0 = time.time()
        ftot, fdiv, rm = O.fast_perft(start, 5, O.REF, threads=th)
        rtot, rdiv = O.ref_perft(cells0, 0, 5, threads=th)
        rd = ref_divide_by_move(rdiv, rm)
        assert rtot == ftot and rd == [int(v) for v in fdiv], ("startpos d5", rtot, ftot)
        out["startpos_d5"] = {"total": ftot, "divide": {str(int(m)): v for m, v in zip(rm, rd)},
                              "engines": ["refcpu", "fastcpu"], "seconds": round(time.time() - t0, 1)}
        save()
        print("startpos d5", ftot, round(time.time() - t0, 1), "s", flush=True)
    # ------------------------------------- two perft(6) subtrees (depth 5 below a root move)
    if "startpos_d6_subtrees" not in out:
        t0 = time.time()
        _, _, rm = O.fast_perft(start, 1, O.REF, threads=th)
        subs = {}
        for m in (int(rm[0]), int(rm[-1])):  # the first and last root moves in fastcpu order (Nb1-a3, h2-h4)
            f, t = m & 63, (m >> 6) & 63
            v, cells, turn, _ = O.ref_apply(cells0, 0, "", f >> 3, f & 7, t >> 3, t & 7)
            assert v == 0
            child = O.fast_make(start, m)
            ftot, _, _ = O.fast_perft(child, 5, O.REF, threads=th)
            rtot, _ = O.ref_perft(cells, turn, 5, threads=th)
            assert rtot == ftot, ("d6 subtree", m, rtot, ftot)
            subs[str(m)] = ftot
            print("d6 subtree", m, ftot, round(time.time() - t0, 1), "s", flush=True)
        out["startpos_d6_subtrees"] = {"divide": subs, "engines": ["refcpu", "fastcpu"],
                                       "seconds": round(time.time() - t0, 1)}
        save()
    # ---------------------------------------------------------- suite FENs at REF d4
    if "suite_d4" not in out:
        t0 = time.time()
        suite = {}
        for name, (fen, _) in FIDE_SUITE.items():
            p = O.Pos.from_fen(fen)
            cnt = {}
            for d in range(1, 5):
                ftot, _, _ = O.fast_perft(p, d, O.REF, threads=th)
                rtot, _ = O.ref_perft(p.cells, p.stm, d, threads=th)
                assert rtot == ftot, (name, d, rtot, ftot)
                cnt[str(d)] = ftot
            suite[name] = {"fen": fen, "perft": cnt}
            print("suite", name, cnt, round(time.time() - t0, 1), "s", flush=True)
        out["suite_d4"] = {"positions": suite, "engines": ["refcpu", "fastcpu"], "seconds": round(time.time() - t0, 1)}
        save()
    # ----------------------------------------------------- random positions at d3
    if "random_d3" not in out:
        t0 = time.time()
        rnd = []
        for p in random_positions(24):
            ftot, _, _ = O.fast_perft(p, 3, O.REF, threads=th)
            rtot, _ = O.ref_perft(p.cells, p.stm, 3, threads=th)
            assert rtot == ftot
            rnd.append({"cells": p.cells.tolist(), "stm": p.stm, "perft3": ftot})
        out["random_d3"] = {"positions": rnd, "engines": ["refcpu", "fastcpu"], "seconds": round(time.time() - t0, 1)}
        save()
        print("random d3 done", round(time.time() - t0, 1), "s", flush=True)
    # ------------------------------------------ fastcpu-only startpos perft(8), perft(9)
    for d in range(8, args.max_depth + 1):
        key = f"startpos_d{d}"
        if key in out:
            continue
        t0 = time.time()
        ftot, fdiv, rm = O.fast_perft(start, d, O.REF, threads=th)
        out[key] = {"total": ftot, "divide": {str(int(m)): int(v) for m, v in zip(rm, fdiv)},
                    "engines": ["fastcpu"], "seconds": round(time.time() - t0, 1)}
        save()
        print(key, ftot, round(time.time() - t0, 1), "s", flush=True)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
