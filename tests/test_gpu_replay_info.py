"""The resync path: dc_replay_info's per-ply move info and dc_history_append's
update_history text (core/src/chess.rs:127-184), on a sample of the C4 games
(BASELINE configs[3] seed), against the literal restatement refcpu, whose
or_ref_apply runs chess.rs's apply_move + update_history one ply at a time."""
import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu
SEED = 0x5EED20241022


def test_replay_info_histories_match_refcpu_on_c4_sample(engine):
    n, plies = 257, 80  # ragged: 4 waves + 1 game
    moves = engine.gen_games(SEED, 0, n, plies, 32)
    bm, dg, info, st = engine.replay_info(moves)
    bm0, dg0, st0 = engine.replay(moves)
    # the info path replays exactly what the plain replay does
    assert np.array_equal(bm, bm0) and np.array_equal(dg, dg0) and st == st0
    words = (n + 63) // 64
    acc = np.zeros((plies, n), bool)
    for w in range(words):
        for b in range(64):
            g = 64 * w + b
            if g < n:
                acc[:, g] = (bm[:, w] >> np.uint64(b)) & np.uint64(1) == 1
    assert np.array_equal(acc, info != 0xFF)
    start = O.startpos_cells()
    for g in range(0, n, 8):  # every 8th game through refcpu (33 games x 80 plies)
        cells, turn, hist = start.copy(), 0, ""
        for p in range(plies):
            m = int(moves[p, g])
            if m == 0xFFFF:
                continue
            f, t = m & 63, (m >> 6) & 63
            v, cells, turn, hist = O.ref_apply(cells, turn, hist, f >> 3, f & 7, t >> 3, t & 7)
            assert (v == 0) == (info[p, g] != 0xFF), (g, p)
        assert dchess.history_append("", moves[:, g], info[:, g]) == hist, g


def test_replay_info_matches_apply_batch_per_ply(engine):
    """info byte per ply == dc_apply_batch's info for the same position and move."""
    n, plies = 128, 40
    moves = engine.gen_games(SEED ^ 7, 5, n, plies, 64)
    _, _, info, _ = engine.replay_info(moves)
    pos = np.array([dchess.startpos()] * n, dchess.POS_DTYPE)
    for p in range(plies):
        mv = moves[p].copy()
        live = mv != 0xFFFF
        new, ver, inf = engine.apply_batch(pos.copy(), np.where(live, mv, 0).astype(np.uint16))
        exp = np.where(live & (ver == 0), inf, 0xFF)
        assert np.array_equal(exp, info[p]), p
        pos = np.where((live & (ver == 0))[:, None], new.view(np.uint8).reshape(n, -1),
                       pos.view(np.uint8).reshape(n, -1)).view(dchess.POS_DTYPE).reshape(n)


def test_replay_info_rejects_fide_and_handles_empty(engine):
    with pytest.raises(dchess.DChessError):
        dchess.lib()  # loaded
        st = dchess._Stats()
        dchess._check(dchess.lib().dc_replay_info(engine.ctx, dchess.RULES_FIDE, None, None, 0, 0, None, None,
                                                  None, None), "dc_replay_info")
    bm, dg, info, st = engine.replay_info(np.zeros((0, 5), np.uint16))
    assert info.shape == (0, 5) and st["validated"] == 0
