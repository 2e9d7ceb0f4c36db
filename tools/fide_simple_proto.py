"""CPU restatement of the FIDE final stage's simple-child split (measurement
and test infrastructure; the kernel is dc_fide_rules.h fide_sens /
fide_for_each_split, used by k_count2b<FideRules> in dc_perft.hip).

For a parent P (side S to move, opponent O) and a legal S move f -> t, the
move is *simple* when it is quiet (t empty; no promotion, castling, en passant
or double push), S is not in check, and neither square is in the sets below
(all set-wise, as the kernel computes them):

  Z'      O's king, its neighbours, and O's back-rank squares b..g while O
          keeps a castling right
  all     Z' | O's slider rays (up to and including the first piece) | O's
          pawn push / double-push / capture squares | for each direction d:
          the open squares seen from Z' toward d that an S slider of d's kind
          also sees looking back, and that slider | the pin segments from O's
          king (first piece O's: up to and including the second piece)
  fsrc    (f only) first pieces seen from Z' toward d with an S slider of d's
          kind behind them, and S pieces first on a line from O's king with
          an O piece second (moving one may pin that piece)
  t_orth / t_diag   (t only, for rook/queen resp. bishop/queen movers) the
          open squares seen from Z' along orthogonal / diagonal lines
  lk, ln, lp        (king / knight / pawn movers) squares from which such an
          S piece attacks Z'
(lines seen from Z' and the S slider rays use the occupancy without O's king,
as O's danger map does.)

Claim: O's legal move count in the child then equals c0 = O's legal move count
in P with O to move and no en-passant square.  `check()` tests the claim
against the oracle (fastcpu) on random descendants of the given roots and
reports the share of simple children.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import oracle_lib as O  # noqa: E402

FULL = (1 << 64) - 1
PIN_PRECISE = os.environ.get("FIDE_PIN_PRECISE") == "1"  # (study) pin segments only where a pin exists
P_, N_, B_, R_, Q_, K_ = range(6)
ORTH = ((1, 0), (-1, 0), (0, 1), (0, -1))
DIAG = ((1, 1), (1, -1), (-1, 1), (-1, -1))
DIRS = ORTH + DIAG
KNIGHT = ((1, 2), (2, 1), (-1, 2), (-2, 1), (1, -2), (2, -1), (-1, -2), (-2, -1))


def bit(s):
    return 1 << s


def sqs(b):
    while b:
        low = b & -b
        yield low.bit_length() - 1
        b ^= low


def on(x, y):
    return 0 <= x < 8 and 0 <= y < 8


def leap_set(src, offs):
    out = 0
    for s in sqs(src):
        x, y = divmod(s, 8)
        for dx, dy in offs:
            if on(x + dx, y + dy):
                out |= bit((x + dx) * 8 + y + dy)
    return out


def fill(src, occ, dirs, stop=True):
    """Squares reached from src along dirs, up to and including the first
    occupied square (stop=False: to the board edge); src itself excluded."""
    out = 0
    for s in sqs(src):
        x, y = divmod(s, 8)
        for dx, dy in dirs:
            a, b = x + dx, y + dy
            while on(a, b):
                out |= bit(a * 8 + b)
                if stop and occ >> (a * 8 + b) & 1:
                    break
                a, b = a + dx, b + dy
    return out


def sets(cells):
    side = [0, 0]
    kind = [[0] * 7 for _ in range(2)]
    for s, c in enumerate(cells):
        if c >= 0:
            side[c >> 3] |= bit(s)
            kind[c >> 3][c & 7] |= bit(s)
    return side, kind


def pawn_att(p, col):
    """Squares attacked by pawns p of colour col (white = 0 moves to +8)."""
    dx = 1 if col == 0 else -1
    return leap_set(p, ((dx, 1), (dx, -1)))


def attacked_by(pos, col, target):
    side, kind = sets(pos.cells)
    occ = side[0] | side[1]
    k = kind[col]
    att = pawn_att(k[P_], col) | leap_set(k[N_], KNIGHT) | leap_set(k[K_], DIRS)
    att |= fill(k[R_] | k[Q_], occ, ORTH) | fill(k[B_] | k[Q_], occ, DIAG)
    return (att & target) != 0


def sens(pos, split_og=False):
    """The kernel's sets (fide_sens) as a dict, or None when no child is simple.
    split_og: O's slider rays and pawn squares left out of "all" and returned
    as "og" (the semi-simple class: only O's slider and pawn moves change)."""
    S, Ot = pos.stm, 1 - pos.stm
    side, kind = sets(pos.cells)
    occ = side[0] | side[1]
    tk, sk = kind[Ot][K_], kind[S][K_]
    if tk == 0 or tk & (tk - 1) or sk == 0 or sk & (sk - 1):
        return None
    if attacked_by(pos, Ot, sk):
        return None  # S in check
    ksq = tk.bit_length() - 1
    zp = tk | leap_set(tk, DIRS)
    if (pos.castle >> (2 * Ot)) & 3:
        zp |= 0x7E << (0 if Ot == 0 else 56)
    occ_nk = occ & ~tk
    e_nk = FULL & ~occ_nk
    s_o, s_d = kind[S][R_] | kind[S][Q_], kind[S][B_] | kind[S][Q_]
    allm, fsrc, t_o, t_d = zp, 0, 0, 0
    for di, d in enumerate(DIRS):
        st = s_o if di < 4 else s_d
        fd = fill(zp, occ_nk, (d,))
        rd = fill(st, occ_nk, ((-d[0], -d[1]),))
        b1 = fd & occ_nk
        if di < 4:
            t_o |= fd & e_nk
        else:
            t_d |= fd & e_nk
        allm |= (fd & rd & e_nk) | (b1 & st)
        fsrc |= b1 & rd
        # pin segment from O's king toward d
        x, y = divmod(ksq, 8)
        ray = []
        a, b = x + d[0], y + d[1]
        while on(a, b):
            ray.append(a * 8 + b)
            a, b = a + d[0], b + d[1]
        blk = [q for q in ray if occ >> q & 1]
        if blk and pos.cells[blk[0]] >> 3 == Ot:
            end = ray.index(blk[1]) + 1 if len(blk) > 1 else len(ray)
            seg = sum(bit(q) for q in ray[:end] if q != blk[0])
            if not PIN_PRECISE or (len(blk) > 1 and st >> blk[1] & 1):
                allm |= seg  # a pin: any change on it can break it
            else:
                # no pin yet: a slider of the line's kind landing past the O piece
                # (before the next piece) makes one, and so can the next piece leaving
                past = sum(bit(q) for q in ray[ray.index(blk[0]) + 1:end] if len(blk) < 2 or q != blk[1])
                if di < 4:
                    t_o |= past
                else:
                    t_d |= past
                if len(blk) > 1:
                    fsrc |= bit(blk[1])
        elif len(blk) > 1 and pos.cells[blk[1]] >> 3 == Ot:
            fsrc |= bit(blk[0])  # an S piece shielding an O piece: moving it may pin that piece
    og = fill(kind[Ot][R_] | kind[Ot][Q_], occ, ORTH) | fill(kind[Ot][B_] | kind[Ot][Q_], occ, DIAG)
    tp = kind[Ot][P_]
    fwd = 8 if Ot == 0 else -8
    shf = (lambda b, n: (b << n) & FULL if n > 0 else b >> -n)
    after1 = 0xFF << 16 if Ot == 0 else 0xFF << 40
    push = shf(tp, fwd)
    og |= push | shf(push & after1, fwd) | pawn_att(tp, Ot)
    if not split_og:
        allm |= og
    return {"all": allm, "fsrc": fsrc, "t_orth": t_o, "t_diag": t_d, K_: leap_set(zp, DIRS),
            N_: leap_set(zp, KNIGHT), P_: pawn_att(zp, Ot), "og": og}


def simple_moves(pos, moves, sn):
    """The legal moves `moves` of pos that are simple under the sets sn."""
    if sn is None:
        return []
    out = []
    for m in moves:
        fr, to, promo = int(m) & 63, (int(m) >> 6) & 63, (int(m) >> 12) & 7
        c = pos.cells[fr] & 7
        if promo or pos.cells[to] >= 0:
            continue
        if c == P_ and ((fr ^ to) & 7 or abs(to - fr) == 16):
            continue  # en passant, double push
        if c == K_ and abs(to - fr) == 2:
            continue  # castling
        sf = sn["all"] | sn["fsrc"] | sn.get(c, 0)
        st = sn["all"] | sn.get(c, 0)
        if c in (R_, Q_):
            st |= sn["t_orth"]
        if c in (B_, Q_):
            st |= sn["t_diag"]
        if sf >> fr & 1 or st >> to & 1:
            continue
        out.append(int(m))
    return out


def check(roots, n_pos, seed=1, dmin=0, dmax=12):
    rng = random.Random(seed)
    tot = simp = bad = 0
    for i in range(n_pos):
        pos = roots[i % len(roots)].copy()
        for _ in range(rng.randrange(dmin, dmax + 1)):
            mv = O.fast_gen_moves(pos, O.FIDE)
            if len(mv) == 0:
                break
            pos = O.fast_make(pos, int(mv[rng.randrange(len(mv))]), O.FIDE)
        moves = O.fast_gen_moves(pos, O.FIDE)
        tot += len(moves)
        sm = simple_moves(pos, moves, sens(pos))
        if not sm:
            continue
        q = pos.copy()
        q.stm, q.ep = 1 - pos.stm, -1
        c0 = len(O.fast_gen_moves(q, O.FIDE))
        for m in sm:
            simp += 1
            if len(O.fast_gen_moves(O.fast_make(pos, m, O.FIDE), O.FIDE)) != c0:
                bad += 1
    return {"positions": n_pos, "children": tot, "simple": simp, "simple_frac": round(simp / max(tot, 1), 4),
            "mismatches": bad}


def main():
    og = json.load(open(os.path.join(HERE, "..", "tests", "golden", "oracle_golden.json")))
    suite = [O.Pos.from_fen(e["fen"]) for e in og["perft_fide"].values()]
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    print(json.dumps({"roots": "startpos, 5 plies", **check([O.Pos()], n, seed=5, dmin=5, dmax=5)}))
    print(json.dumps({"roots": "suite, 0-12 plies", **check(suite, n, seed=1)}))


if __name__ == "__main__":
    main()
