"""CPU check of the final stage's group-wise recount identity (c2c_group's
second queue, dc_ref.h ref_count_child_diag).

For a parent P (side S to move, opponent O) and an S move f -> t whose
squares are off O's orthogonal group (O's rook/queen rays up to and including
the first blocker, and O's rooks/queens themselves), the kernel counts the
child's O moves as

    base(P) - diag(P) + diag(child) + pawns(child)
      + [t held an O piece] (O knights/kings attacking t - the captured
                             knight's or king's own moves in P)

where base = O's knight, king and slider moves and diag = the bishop/queen
diagonal share.  Here every term is evaluated by a plain square-walk
restatement of the REF rules (chess.rs:199-360) and the left side by refcpu
(oracle, ref_perft depth 1 of the child), over random positions that include
several kings and the unknown kind -- the same mix as the GPU's odd-position
perft test.  This pins the algebra; the GPU goldens pin the kernel.
"""
import numpy as np

import oracle_lib as O

P_, N_, B_, R_, Q_, K_, X_ = range(7)  # cells kinds (colour * 8 + kind)
ORTH = ((1, 0), (-1, 0), (0, 1), (0, -1))
DIAG = ((1, 1), (1, -1), (-1, 1), (-1, -1))
KNIGHT = ((1, 2), (2, 1), (-1, 2), (-2, 1), (1, -2), (2, -1), (-1, -2), (-2, -1))
KING = ORTH + DIAG


def colour(c):
    return -1 if c < 0 else c >> 3


def kind(c):
    return -1 if c < 0 else c & 7


def on(x, y):
    return 0 <= x < 8 and 0 <= y < 8


def rays(cells, sq, dirs):
    """Squares a slider on sq reaches: up to and including the first occupied."""
    out = []
    x, y = divmod(sq, 8)
    for dx, dy in dirs:
        a, b = x + dx, y + dy
        while on(a, b):
            out.append(a * 8 + b)
            if cells[a * 8 + b] >= 0:
                break
            a, b = a + dx, b + dy
    return out


def leaps(sq, offs):
    x, y = divmod(sq, 8)
    return [(x + dx) * 8 + y + dy for dx, dy in offs if on(x + dx, y + dy)]


def not_own(cells, s, side):
    return colour(cells[s]) != side


def group_counts(cells, side):
    """(knights + kings, orthogonal, diagonal) move counts and the orth mask."""
    nk = orth = diag = 0
    omask = set()
    for sq in range(64):
        c = cells[sq]
        if colour(c) != side:
            continue
        k = kind(c)
        if k == N_:
            nk += sum(not_own(cells, s, side) for s in leaps(sq, KNIGHT))
        elif k == K_:
            nk += sum(not_own(cells, s, side) for s in leaps(sq, KING))
        if k in (R_, Q_):
            r = rays(cells, sq, ORTH)
            orth += sum(not_own(cells, s, side) for s in r)
            omask.update(r)
            omask.add(sq)
        if k in (B_, Q_):
            diag += sum(not_own(cells, s, side) for s in rays(cells, sq, DIAG))
    return nk, orth, diag, omask


def pawn_count(cells, side):
    n = 0
    d = 1 if side == 0 else -1
    start = 1 if side == 0 else 6
    for sq in range(64):
        if colour(cells[sq]) != side or kind(cells[sq]) != P_:
            continue
        x, y = divmod(sq, 8)
        if on(x + d, y) and cells[(x + d) * 8 + y] < 0:
            n += 1
            if x == start and cells[(x + 2 * d) * 8 + y] < 0:
                n += 1
        for dy in (-1, 1):
            if on(x + d, y + dy):
                c = cells[(x + d) * 8 + y + dy]
                if c >= 0 and colour(c) != side:
                    n += 1
    return n


def group_wise(cells, side, f, t):
    nk, orth, diag_p, _ = group_counts(cells, side)
    base = nk + orth + diag_p
    ch = cells.copy()
    ch[t], ch[f] = ch[f], -1
    _, _, diag_c, _ = group_counts(ch, side)
    c = base - diag_p + diag_c + pawn_count(ch, side)
    if colour(cells[t]) == side:  # capture of an O piece
        gain = sum(colour(ch[s]) == side and kind(ch[s]) == N_ for s in leaps(t, KNIGHT))
        gain += sum(colour(ch[s]) == side and kind(ch[s]) == K_ for s in leaps(t, KING))
        lost = 0
        if kind(cells[t]) == N_:
            lost = sum(not_own(cells, s, side) for s in leaps(t, KNIGHT))
        elif kind(cells[t]) == K_:
            lost = sum(not_own(cells, s, side) for s in leaps(t, KING))
        c += gain - lost
    return c


def random_cells(rng, n):
    cells = np.full(64, -1, np.int8)
    sq = rng.choice(64, n, replace=False)
    cells[sq] = rng.integers(0, 2, n) * 8 + rng.integers(0, 7, n)
    return cells


def test_group_wise_recount_matches_refcpu():
    rng = np.random.default_rng(31)
    checked = captures = 0
    positions = [O.startpos_cells()] + [random_cells(rng, int(rng.integers(6, 26))) for _ in range(60)]
    for cells in positions:
        for stm in (0, 1):
            side = 1 - stm
            _, _, _, omask = group_counts(cells, side)
            ok = np.nonzero(O.ref_verdicts_all(cells, stm) == 0)[0]
            for idx in ok.tolist():
                f, t = idx >> 6, idx & 63
                if f in omask or t in omask:
                    continue  # the full-recount queue
                ch = cells.copy()
                ch[t], ch[f] = ch[f], -1
                want = O.ref_perft(ch, side, 1)[0]
                assert group_wise(cells, side, f, t) == want, (cells.tolist(), stm, f, t)
                checked += 1
                captures += colour(cells[t]) == side
    assert checked > 500 and captures > 50
