"""CPU tests: the oracle against the reference's own known answers.

refcpu is the literal restatement of /root/reference/core/src/chess.rs; the
entries of tests/golden/known_answers.json marked ref_test are the reference's
unit tests (chess.rs:504-556), the rest are SURVEY Appendix C vectors.
fastcpu is checked for equivalence with refcpu over all 4096 (from,to) pairs.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KA = json.load(open(os.path.join(GOLD, "known_answers.json")))
OG = json.load(open(os.path.join(GOLD, "oracle_golden.json")))


@pytest.mark.parametrize("case", KA["validate"], ids=lambda c: f"ka{c['id']}")
def test_refcpu_known_answers(case):
    s = O.startpos_cells()
    v = O.ref_validate(s, case["turn"], *case["from"], *case["to"])
    assert v == case["verdict"]


def test_refcpu_messages_match_reference_strings():
    # chess.rs:104-106, :113-115, :119-121
    assert O.ref_message(1) == "No piece at the source location"
    assert O.ref_message(2) == "It's not this piece's turn to move"
    assert O.ref_message(3) == "Invalid move for the piece"


def test_refcpu_apply_history_sequence():
    seq = KA["apply_sequence"]
    cells, turn, hist = O.startpos_cells(), 0, ""
    for (f, t), want in zip(seq["moves"], seq["verdicts"]):
        v, cells, turn, hist = O.ref_apply(cells, turn, hist, *f, *t)
        assert v == want
    assert hist == seq["history"]
    assert turn == seq["turn"]


def test_refcpu_rejected_apply_leaves_state():
    cells = O.startpos_cells()
    v, c2, t2, h2 = O.ref_apply(cells, 0, "", 0, 0, 2, 2)
    assert v == O.ILLEGAL and (c2 == cells).all() and t2 == 0 and h2 == ""


def test_fast_matches_ref_on_known_answers():
    p = O.Pos()
    for case in KA["validate"]:
        (fx, fy), (tx, ty) = case["from"], case["to"]
        q = p.copy()
        q.stm = case["turn"]
        m = 0x8000 if max(fx, fy, tx, ty) >= 8 else (8 * fx + fy) | ((8 * tx + ty) << 6)
        assert O.fast_validate(q, m, O.REF) == case["verdict"], case


def _random_positions(n, seed):
    mv = O.fast_gen_games(seed, 0, n, 70, noise_per_256=0)
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n):
        p = O.Pos()
        for ply in range(int(rng.integers(0, 70))):
            m = int(mv[ply, g])
            if m == O.SENTINEL:
                break
            if O.fast_validate(p, m) == O.OK:
                p = O.fast_make(p, m)
        out.append(p)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fast_equals_ref_all_pairs(seed):
    """fastcpu RULES_REF == refcpu over every (from,to) pair, both sides to move."""
    for p in _random_positions(12, seed):
        for stm in (0, 1):
            q = p.copy()
            q.stm = stm
            a = O.fast_verdicts_all(q, O.REF)
            b = O.ref_verdicts_all(q.cells, stm)
            assert (a == b).all()


def test_odd_pieces_all_pairs():
    """Unknown-kind pieces (kind 'X') block, are capturable and never move (chess.rs:210)."""
    rng = np.random.default_rng(7)
    for _ in range(8):
        cells = np.full(64, -1, np.int8)
        sq = rng.choice(64, 20, replace=False)
        cells[sq] = rng.integers(0, 2, 20) * 8 + rng.integers(0, 7, 20)
        for stm in (0, 1):
            p = O.Pos(cells, stm, 0, -1)
            assert (O.fast_verdicts_all(p, O.REF) == O.ref_verdicts_all(cells, stm)).all()


def test_perft_ref_startpos_shallow():
    s = O.startpos_cells()
    for d, want in KA["perft_ref_startpos_shallow"].items():
        if d == "why":
            continue
        assert O.ref_perft(s, 0, int(d), threads=8)[0] == want
        assert O.fast_perft(O.Pos(), int(d), O.REF)[0] == want


def test_perft_ref_golden_fast():
    for d in range(1, 6):
        tot, div, rm = O.fast_perft(O.Pos(), d, O.REF)
        g = OG["perft_ref"]["startpos"][str(d)]
        assert tot == g["total"]
        assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]


def test_perft_ref_random_positions_golden():
    for e in OG["perft_ref"]["random_positions"][:8]:
        p = O.Pos(np.array(e["cells"], np.int8), e["stm"], 0, -1)
        for d in ("1", "2", "3"):
            assert O.fast_perft(p, int(d), O.REF)[0] == e["perft"][d]


@pytest.mark.parametrize("name", ["startpos", "kiwipete", "pos3", "pos4", "pos5", "pos6"])
def test_perft_fide_published(name):
    e = OG["perft_fide"][name]
    p = O.Pos.from_fen(e["fen"])
    depth = 3 if name in ("kiwipete", "pos5", "pos6") else 4
    for d in range(1, depth + 1):
        assert O.fast_perft(p, d, O.FIDE)[0] == e["perft"][str(d)]


def test_games_fixture_and_ref_replay():
    import hashlib
    g = OG["games"]
    mv = O.fast_gen_games(g["seed"], g["first_game"], g["n_games"], g["n_plies"], g["noise_per_256"])
    assert hashlib.sha256(mv.tobytes()).hexdigest() == g["moves_sha256"]
    bm, dg, st = O.ref_replay(mv, threads=8)
    assert hashlib.sha256(bm.tobytes()).hexdigest() == g["bitmap_sha256"]
    assert hashlib.sha256(dg.tobytes()).hexdigest() == g["digests_sha256"]
    assert int(st[0]) == g["stats"]["validated"] and int(st[1]) == g["stats"]["accepted"]
    fbm, fdg, fst = O.fast_replay(mv)
    assert (fbm == bm).all() and (fdg == dg).all() and (fst == st).all()


def test_replay_properties():
    mv = O.fast_gen_games(99, 5, 130, 50, noise_per_256=64)
    bm, dg, st = O.fast_replay(mv)
    # size-independent invariants: accepted = popcount(bitmap), validated = non-sentinel plies
    assert int(st[1]) == int(sum(bin(int(w)).count("1") for w in bm.ravel()))
    assert int(st[0]) == int((mv != O.SENTINEL).sum())
    assert int(st[0]) == int(st[1]) + int(st[2])
    x = 0
    for d in dg:
        x ^= int(d)
    assert x == int(st[4])
    assert int(dg.astype(np.uint64).sum(dtype=np.uint64)) == int(st[3])


def test_startpos_quad_golden():
    assert [int(x) for x in O.quad(O.startpos_cells())] == OG["startpos_quad"]


REF_D6 = json.load(open(os.path.join(GOLD, "ref_d6.json")))["positions"]


@pytest.mark.parametrize("name", sorted(REF_D6))
def test_ref_d6_golden_consistent(name):
    """tests/golden/ref_d6.json (REF perft(6) off the startpos tree): the divide
    sums to the total, the root moves are fastcpu's, and refcpu (the literal
    chess.rs restatement) agrees with fastcpu at depth 2 of the same board."""
    e = REF_D6[name]
    p = O.Pos(np.array(e["cells"], np.int8), e["stm"], 0, -1)
    assert sum(e["divide"].values()) == e["total"]
    _, _, rm = O.fast_perft(p, 1, O.REF, threads=2)
    assert sorted(str(int(m)) for m in rm) == sorted(e["divide"])
    ft, _, _ = O.fast_perft(p, 2, O.REF, threads=2)
    rt, _ = O.ref_perft(p.cells, p.stm, 2, threads=2)
    assert ft == rt
