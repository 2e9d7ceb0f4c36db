#!/usr/bin/env python3
"""Prototype of the REF final stage's target-side pawn correction (k_count3c,
dc_ref.h ref_parent_split).

Round 4's split counts a child in bulk (count_O = base + pawn_O of the parent,
never enumerated) when the move is quiet and both f and t are off att (O's
slider rays) and off G (O's pawn-sensitive squares).  The quiet moves with f or
t in G were enumerated and their pawn term recounted per child.  Here a quiet
move with f off att and G and t off att is counted in bulk too, with the pawn
term corrected by g(t):

    g(t) = [t in cw] + [t in ce] - [t in q1] - [t in mid] - [t in land]

on the parent (cw/ce: O pawn capture squares, q1: O push squares, mid: middle
squares of an O double push whose landing is empty, land: landings whose
middle is empty).  Squares with |g| = 2 stay enumerated, so the kernel needs
two planes: g = +1 (P1) and g = -1 (N1).

Checks the identity count_O(P o m) = base + pawn_O(P) + g(t) against the oracle
on random REF positions (descendants of startpos and of random mid-game
boards) and prints how many children move from the enumerated set to the bulk.
usage: ref_gsplit_proto.py [n_positions]"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import oracle_lib as O  # noqa: E402

P_, N_, B_, R_, Q_, K_ = range(6)
FULL = (1 << 64) - 1
NOT_A = FULL ^ 0x0101010101010101
NOT_H = FULL ^ 0x8080808080808080


def sh(x, s):
    return (x << s) & FULL if s >= 0 else x >> -s


def bits(cells, pred):
    b = 0
    for s in range(64):
        if cells[s] >= 0 and pred(int(cells[s])):
            b |= 1 << s
    return b


def ray(src, empty, s, m):
    """squares reached from src toward s (first blocker included), guard mask m."""
    out = 0
    g = src
    while g:
        g = sh(g, s) & m
        out |= g
        g &= empty
    return out


DIRS_O = ((8, FULL), (-8, FULL), (1, NOT_A), (-1, NOT_H))
DIRS_D = ((9, NOT_A), (-9, NOT_H), (7, NOT_H), (-7, NOT_A))


def planes(pos):
    """att, G, P1, N1, P2N2 of the parent for O = 1 - stm."""
    c = pos.cells
    o = 1 - pos.stm
    occ = bits(c, lambda v: True)
    empty = FULL ^ occ
    ownO = bits(c, lambda v: v >> 3 == o)
    PO = bits(c, lambda v: v >> 3 == o and v & 7 == P_)
    OO = bits(c, lambda v: v >> 3 == o and v & 7 in (R_, Q_))
    DO = bits(c, lambda v: v >> 3 == o and v & 7 in (B_, Q_))
    att = 0
    for s, m in DIRS_O:
        att |= ray(OO, empty, s, m)
    for s, m in DIRS_D:
        att |= ray(DO, empty, s, m)
    F = 8 if o == 0 else -8
    row_dbl = 0xFF << (24 if o == 0 else 32)   # landing row of a double push
    row_mid = 0xFF << (16 if o == 0 else 40)   # its middle row
    q1 = sh(PO, F)
    cw = sh(PO & NOT_A, F - 1) if True else 0   # toward file a
    ce = sh(PO & NOT_H, F + 1)
    push1 = q1 & empty
    land = sh(push1, F) & row_dbl
    mid = q1 & row_mid & sh(empty & row_dbl, -F)
    G = q1 | cw | ce | land
    pos_w = [(cw >> s & 1) + (ce >> s & 1) for s in range(64)]
    neg_w = [(q1 >> s & 1) + (mid >> s & 1) + (land >> s & 1) for s in range(64)]
    g = [pos_w[s] - neg_w[s] for s in range(64)]
    P1 = sum(1 << s for s in range(64) if g[s] == 1)
    N1 = sum(1 << s for s in range(64) if g[s] == -1)
    big = sum(1 << s for s in range(64) if abs(g[s]) >= 2)
    mids = q1 & row_mid  # middle squares of O double pushes (an O pawn on its start row behind)
    return dict(att=att, G=G, P1=P1, N1=N1, big=big, g=g, occ=occ, ownO=ownO, mids=mids, F=F)


def count_o(pos):
    q = pos.copy()
    q.stm = 1 - pos.stm
    return len(O.fast_gen_moves(q, O.REF))


def check(n, seed=3):
    rng = random.Random(seed)
    import json
    import numpy as np
    d6 = json.load(open(os.path.join(HERE, "..", "tests", "golden", "ref_d6.json")))["positions"]
    # startpos and the REF d6 goldens' boards (mid-game, kingless, unknown-kind, two kings)
    roots = [O.Pos()] + [O.Pos(np.array(e["cells"], np.int8), e["stm"], 0, -1) for e in d6.values()]
    st = dict(positions=0, children=0, simple_old=0, bulk_new=0, quiet_special_old=0, quiet_special_new=0,
              big_targets=0, mismatches=0, src_bulk=0, src_mismatches=0, quiet_special_src=0)
    for i in range(n):
        pos = roots[0 if i % 2 else rng.randrange(len(roots))].copy()
        for _ in range(rng.choice([5, 5, 5, 9, 15, 25]) if i % 2 else rng.randrange(0, 6)):
            mv = O.fast_gen_moves(pos, O.REF)
            if len(mv) == 0:
                break
            pos = O.fast_make(pos, int(mv[rng.randrange(len(mv))]), O.REF)
        moves = O.fast_gen_moves(pos, O.REF)
        if len(moves) == 0:
            continue
        st["positions"] += 1
        pl = planes(pos)
        att, G = pl["att"], pl["G"]
        base_pawn = count_o(pos)  # base + pawn_O: O's count in the parent with O to move
        for m in moves:
            m = int(m)
            f, t = m & 63, (m >> 6) & 63
            st["children"] += 1
            quiet = not (pl["occ"] >> t & 1) and not (att >> f & 1) and not (att >> t & 1)
            if not quiet:
                continue
            old_simple = not (G >> f & 1) and not (G >> t & 1)
            new_bulk = not (G >> f & 1) and not (pl["big"] >> t & 1)
            st["simple_old"] += old_simple
            st["bulk_new"] += new_bulk
            st["quiet_special_old"] += not old_simple
            st["quiet_special_new"] += not new_bulk
            st["big_targets"] += bool(not (G >> f & 1) and pl["big"] >> t & 1)
            # source side (round 5b): a pawn, knight or king on G (off BIG) moving quietly to t off BIG:
            # count_O = base + pawn_O + g(t) - g(f) + I, I = -1 when f, t are the mid and landing
            # squares of one O double push
            kind = int(pos.cells[f]) & 7
            src_bulk = (G >> f & 1) and not (pl["big"] >> f & 1) and not (pl["big"] >> t & 1) and kind in (P_, N_, K_)
            if src_bulk:
                mids, F = pl["mids"], pl["F"]
                pair = (mids >> f & 1 and t == f + F) or (mids >> t & 1 and f == t + F)
                want = len(O.fast_gen_moves(O.fast_make(pos, m, O.REF), O.REF))
                got = base_pawn + pl["g"][t] - pl["g"][f] - (1 if pair else 0)
                st["src_bulk"] += 1
                if want != got:
                    st["src_mismatches"] += 1
                    if st["src_mismatches"] < 5:
                        print("src mismatch", pos.cells.tolist(), pos.stm, f, t, want, got, file=sys.stderr)
            elif not new_bulk:
                st["quiet_special_src"] += 1
            if new_bulk:
                want = len(O.fast_gen_moves(O.fast_make(pos, m, O.REF), O.REF))  # O to move in the child
                got = base_pawn + pl["g"][t]
                if want != got:
                    st["mismatches"] += 1
                    if st["mismatches"] < 5:
                        print("mismatch", pos.cells.tolist(), pos.stm, f, t, want, got, file=sys.stderr)
    return st


if __name__ == "__main__":
    print(check(int(sys.argv[1]) if len(sys.argv) > 1 else 400))
