"""REF perft(6) pins off the startpos tree -- TEST INFRASTRUCTURE.

Run:  python tests/golden/make_ref_d6_golden.py [--threads 8]     (~5 min on 8 cores)

The GPU's full-occupancy final stage (k_count3c, the last three plies) was
pinned at depth >= 6 only on startpos-derived trees.  This script pins REF
perft(6), with the per-root-move divide, of
  * the six standard-suite FENs (castling / en-passant fields carried, ignored
    by the reference's rules, /root/reference/core/src/chess.rs:199-360), and
  * ten mid-game positions reached by seeded REF games, four of them edited into
    boards the reference accepts but startpos never reaches: no white king, no
    kings at all, an unknown-kind piece (chess.rs:203-211: never moves, blocks,
    can be captured), two white kings (chess.rs:350-360 has no king count);
by fastcpu (the mailbox engine), and cross-checks each position with refcpu --
the literal restatement of chess.rs, every (from,to) pair through
validate_move -- on one subtree: the depth-4 subtree below the first root
move's first reply, in fastcpu's canonical order.

Output: tests/golden/ref_d6.json.
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

UNKNOWN = 6  # fastcpu kind X: a piece kind the reference's can_move_to does not know


def edited_positions():
    """Ten mid-game REF positions; the last four edited (see the module doc)."""
    ps = random_positions(10, seed=20241022, plies=(16, 48))
    out = []
    for i, p in enumerate(ps):
        c = p.cells.copy()
        note = "random game"
        if i == 6:
            c[c == 5] = -1  # white king gone
            note = "no white king"
        elif i == 7:
            c[(c == 5) | (c == 13)] = -1
            note = "no kings"
        elif i == 8:
            empty = np.nonzero(c < 0)[0]
            c[empty[len(empty) // 2]] = 8 + UNKNOWN
            c[empty[len(empty) // 3]] = UNKNOWN
            note = "two unknown-kind pieces (one each side)"
        elif i == 9:
            empty = np.nonzero(c < 0)[0]
            c[empty[len(empty) // 2]] = 5
            note = "two white kings"
        out.append((f"mid{i}", O.Pos(c, p.stm, 0, -1), note))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=os.path.join(HERE, "ref_d6.json"))
    args = ap.parse_args()
    th = args.threads
    items = [(name, O.Pos.from_fen(fen), "suite FEN " + fen) for name, (fen, _) in FIDE_SUITE.items()]
    items += edited_positions()
    out = {"engines": "fastcpu perft(6) with divide; refcpu == fastcpu on each position's depth-4 subtree "
                      "below its first root move's first reply", "positions": {}}
    for name, p, note in items:
        t0 = time.time()
        tot, div, rm = O.fast_perft(p, 6, O.REF, threads=th)
        # refcpu cross-check on one subtree
        m1 = int(rm[0])
        c1 = O.fast_make(p, m1)
        _, _, rm1 = O.fast_perft(c1, 1, O.REF, threads=th)
        sub = {"path": [m1]}
        if len(rm1):
            m2 = int(rm1[0])
            c2 = O.fast_make(c1, m2)
            ft, _, _ = O.fast_perft(c2, 4, O.REF, threads=th)
            rt, _ = O.ref_perft(c2.cells, c2.stm, 4, threads=th)
            assert rt == ft, (name, rt, ft)
            sub = {"path": [m1, m2], "depth": 4, "total": ft}
        out["positions"][name] = {"note": note, "cells": p.cells.tolist(), "stm": int(p.stm),
                                  "castle": int(p.castle), "ep": int(p.ep), "total": int(tot),
                                  "divide": {str(int(m)): int(v) for m, v in zip(rm, div)},
                                  "refcpu_subtree": sub, "seconds": round(time.time() - t0, 1)}
        print(name, note, tot, round(time.time() - t0, 1), "s", flush=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
