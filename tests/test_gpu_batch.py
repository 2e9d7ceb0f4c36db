"""GPU tests of the batch perft (dc_perft_batch / dc_perft_batch_repeat_device):
several root positions with the same side to move counted as one tree, their
root moves sharing the divide tags (dc_api.hip; k_expand_top stages up to
DC_PERFT_BATCH_MAX roots).  Pinned by the published FIDE suite tables
(tests/golden/oracle_golden.json) and, per root move, by the single-position
perft of the same build and by fastcpu."""
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu

OG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))["perft_fide"]
SUITE = ["kiwipete", "pos3", "pos4", "pos5", "pos6", "startpos"]  # all white to move: one batch
FIDE, REF = dchess.RULES_FIDE, dchess.RULES_REF
W = 258


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5])
def test_fide_suite_batch_published(engine, depth):
    pos = [dchess.pos_from_fen(OG[k]["fen"]) for k in SUITE]
    tot, div, rm, rp = engine.perft_batch(pos, depth, rules=FIDE)
    assert [int(x) for x in tot] == [OG[k]["perft"][str(depth)] for k in SUITE]
    # the concatenated divide is each position's own divide, in position order
    k = 0
    for i, p in enumerate(pos):
        t1, d1, r1 = engine.perft(p, depth, rules=FIDE)
        n = len(r1)
        assert (rp[k:k + n] == i).all()
        assert (rm[k:k + n] == r1).all() and (div[k:k + n] == d1).all()
        k += n
    assert k == len(rm)


def test_ref_batch_random_positions(engine):
    # REF positions of one side to move (random legal games of even length), some kingless
    mv = O.fast_gen_games(77, 0, 64, 40, noise_per_256=0, rules=O.REF)
    rng = np.random.default_rng(5)
    ps = []
    for g in range(64):
        p = O.Pos()
        for ply in range(2 * int(rng.integers(0, 20))):
            m = int(mv[ply, g])
            if m == O.SENTINEL or O.fast_validate(p, m, O.REF) != O.OK:
                break
            p = O.fast_make(p, m, O.REF)
        if p.stm == 0:
            ps.append(p)
    ps = ps[:7]
    pos = [dchess.pos_from_cells(p.cells, p.stm) for p in ps]
    for depth in (2, 3, 4):
        tot, div, rm, rp = engine.perft_batch(pos, depth, rules=REF)
        for i, p in enumerate(ps):
            assert int(tot[i]) == O.fast_perft(p, depth, O.REF)[0], (i, depth)
            assert int(div[rp == i].sum()) == int(tot[i])


def test_batch_repeat_device_records(engine):
    pos = [dchess.pos_from_fen(OG[k]["fen"]) for k in SUITE]
    tot, div, rm, rp = engine.perft_batch(pos, 4, rules=FIDE)
    runs = 10  # one 8-run batch graph and two single runs
    buf = engine.alloc(runs * W * 8)
    engine.perft_batch_repeat_device(pos, 4, 3, runs, buf, rules=FIDE)
    engine.synchronize()
    res = buf.download(np.uint64, runs * W).reshape(runs, W)
    buf.free()
    for r in range(runs):
        assert int(res[r, 257]) == int(tot.sum())
        assert (res[r, :len(div)] == div).all()
        per = [int(res[r, :len(div)][rp == i].sum()) for i in range(len(pos))]
        assert per == [OG[k]["perft"]["4"] for k in SUITE]


def test_batch_argument_errors(engine):
    p = dchess.startpos()
    with pytest.raises(dchess.DChessError):
        engine.perft_batch([], 3)
    with pytest.raises(dchess.DChessError):
        engine.perft_batch([p] * 9, 3)  # past DC_PERFT_BATCH_MAX
    q = np.array([p], dchess.POS_DTYPE)[0]
    q["stm"] = 1
    with pytest.raises(dchess.DChessError):
        engine.perft_batch([p, q], 3)  # mixed side to move
    # more than 256 root moves in all: the top kernel flags it
    kiwi = dchess.pos_from_fen(OG["kiwipete"]["fen"])
    with pytest.raises(dchess.DChessError):
        engine.perft_batch([kiwi] * 6, 2, rules=FIDE)  # 6 x 48 = 288 root moves
