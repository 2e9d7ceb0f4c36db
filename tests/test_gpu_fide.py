"""GPU parity tests for RULES_FIDE (standard chess: castling, en passant,
promotion, no self-check).  The reference validator does not implement these
rules, so the pins are the published perft tables
(tests/golden/oracle_golden.json "perft_fide") and the independent fastcpu
mailbox engine."""
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu

OG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
FIDE = dchess.RULES_FIDE
DEPTHS = {"startpos": 5, "kiwipete": 5, "pos3": 5, "pos4": 5, "pos5": 5, "pos6": 5}  # C3: the suite at depth 5


def dpos(p):
    d = dchess.pos_from_cells(p.cells, p.stm)
    d["castle"], d["ep"] = p.castle, p.ep
    return d


@pytest.mark.parametrize("name", list(DEPTHS))
def test_perft_suite_published(engine, name):
    e = OG["perft_fide"][name]
    pos = dchess.pos_from_fen(e["fen"])
    for d in range(1, DEPTHS[name] + 1):
        tot, div, rm = engine.perft(pos, d, rules=FIDE)
        assert tot == e["perft"][str(d)], (name, d)
        if d <= 3:
            ot, od, orm = O.fast_perft(O.Pos.from_fen(e["fen"]), d, O.FIDE)
            assert dict(zip(rm.tolist(), div.tolist())) == dict(zip(orm.tolist(), od.tolist()))


def _fide_positions(n, seed):
    mv = O.fast_gen_games(seed, 0, n, 120, noise_per_256=0, rules=O.FIDE)
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n):
        p = O.Pos()
        for ply in range(int(rng.integers(0, 120))):
            m = int(mv[ply, g])
            if m == O.SENTINEL:
                break
            if O.fast_validate(p, m, O.FIDE) == O.OK:
                p = O.fast_make(p, m, O.FIDE)
        out.append(p)
    # plus the suite positions (castling / ep / promotion rich)
    out += [O.Pos.from_fen(e["fen"]) for e in OG["perft_fide"].values()]
    return out


def test_perft_random_fide_positions(engine):
    for p in _fide_positions(24, 31):
        for d in (1, 2, 3):
            assert engine.perft(dpos(p), d, rules=FIDE)[0] == O.fast_perft(p, d, O.FIDE)[0]


def test_validate_all_pairs_fide(engine):
    ps = _fide_positions(20, 41)
    base = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    pos, moves, want = [], [], []
    for p in ps:
        legal = O.fast_gen_moves(p, O.FIDE)
        extra = np.array(sorted(set(int(m) for m in legal if m >> 12)) + [int(m) ^ (1 << 12) for m in legal if m >> 12]
                         + [0x8000], np.uint16)
        mv = np.concatenate([base, extra])
        pos.append(np.repeat(np.array([dpos(p)], dchess.POS_DTYPE), len(mv)))
        moves.append(mv)
        want.append(np.array([O.fast_validate(p, int(m), O.FIDE) for m in mv], np.uint8))
    got = engine.validate_batch(np.concatenate(pos), np.concatenate(moves), rules=FIDE)
    assert (got == np.concatenate(want)).all()


def test_apply_fide_vs_oracle(engine):
    ps = _fide_positions(40, 51)
    pos, moves, exp = [], [], []
    for p in ps:
        for m in O.fast_gen_moves(p, O.FIDE)[:12]:
            pos.append(dpos(p))
            moves.append(int(m))
            exp.append(dpos(O.fast_make(p, int(m), O.FIDE)))
    new, ver, _ = engine.apply_batch(np.array(pos, dchess.POS_DTYPE), np.array(moves, np.uint16), rules=FIDE)
    e = np.array(exp, dchess.POS_DTYPE)
    assert (ver == 0).all()
    assert (new["bb"] == e["bb"]).all() and (new["stm"] == e["stm"]).all()
    assert (new["castle"] == e["castle"]).all() and (new["ep"] == e["ep"]).all()


def test_gen_and_replay_fide(engine):
    mv = engine.gen_games(777, 10, 300, 120, 32, rules=FIDE)
    omv = O.fast_gen_games(777, 10, 300, 120, noise_per_256=32, rules=O.FIDE)
    assert (mv == omv).all()
    bm, dg, st = engine.replay(mv, rules=FIDE)
    fbm, fdg, fst = O.fast_replay(mv, rules=O.FIDE)
    assert (bm == fbm).all() and (dg == fdg).all() and st["accepted"] == int(fst[1])


def test_perft7_startpos_fide(engine):
    """SURVEY §8d C5 (FIDE half) on one GPU: published 3,195,901,860."""
    assert engine.perft(dchess.startpos(), 7, rules=FIDE)[0] == OG["perft_fide"]["startpos"]["perft"]["7"]


@pytest.mark.parametrize("name,depth", [("startpos", 8), ("kiwipete", 6), ("pos3", 7), ("pos4", 6), ("pos6", 6)])
def test_perft_fide_deep_published(engine, name, depth):
    """FIDE past depth 7 and past the suite's depth 5, through the BFS levels
    (startpos d8: ply 6 = 119M boards, 4.3 GB, then the final stage's two
    plies): the published chessprogramming-wiki counts."""
    e = OG["perft_fide"][name]
    assert engine.perft(dchess.pos_from_fen(e["fen"]), depth, rules=FIDE)[0] == e["perft"][str(depth)]


@pytest.mark.parametrize("depth,n_shards,split", [(6, 3, 4), (6, 2, 3)])
def test_perft_startpos_fide_shards(engine, depth, n_shards, split):
    """FIDE through the same front end (k_make_count with FideRules, strided
    shards cut at ply 3 or 4): the shards sum to the published perft."""
    t = sum(engine.perft_shard(dchess.startpos(), depth, split, k, n_shards, rules=FIDE)[0] for k in range(n_shards))
    assert t == OG["perft_fide"]["startpos"]["perft"][str(depth)]
