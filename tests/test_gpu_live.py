"""The live validator (dc_live_validator): small validate / apply calls served by
one resident wave through the stamped mailbox (dc_kernels.h LiveBox) must give
exactly what the launched path and the oracle give -- the reference's
validate_move / apply_move (core/src/chess.rs:43-125) as called by
is_valid_tx (core/src/consensus/hotstuff.rs:138) and commit_block (:52)."""
import time

import numpy as np
import pytest

import dchess
import oracle_lib as O
from test_gpu_fide import _fide_positions, dpos
from test_gpu_ref import _positions, pos_of

pytestmark = pytest.mark.gpu

FIDE = dchess.RULES_FIDE


@pytest.fixture(scope="module")
def live():
    e = dchess.Engine(0)
    e.live_validator(200_000)
    yield e
    e.live_validator(0)
    e.close()


def _pool(seed):
    ps = _positions(8, seed)
    all_moves = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    pool_pos, pool_want = [], []
    for p in ps:
        for stm in (0, 1):
            q = p.copy()
            q.stm = stm
            pool_pos.append(np.repeat(np.array([pos_of(q)], dchess.POS_DTYPE), 4096))
            pool_want.append(O.ref_verdicts_all(q.cells, stm))
    return np.concatenate(pool_pos), np.tile(all_moves, len(pool_want)), np.concatenate(pool_want)


def test_live_batch_sizes_across_paths(live):
    """n either side of the live path's 64 (65 and up take the launched path),
    back to back: verdicts equal the literal restatement's, apply agrees."""
    pool_pos, pool_mv, pool_want = _pool(21)
    rng = np.random.default_rng(22)
    for n in (1, 2, 63, 64, 65, 1, 64, 256, 1, 3, 1):
        idx = rng.choice(len(pool_mv), n, replace=False)
        assert (live.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all(), n
        newpos, v, _ = live.apply_batch(pool_pos[idx], pool_mv[idx])
        assert (v == pool_want[idx]).all(), n
        moved = v == 0
        assert (newpos["stm"][moved] != pool_pos[idx]["stm"][moved]).all()
        assert (newpos[~moved] == pool_pos[idx][~moved]).all()


def test_live_apply_matches_launched(live, engine):
    """Positions, verdicts and the history info byte through the mailbox equal
    the launched kernel's (k_apply_ref) for accepted and rejected moves."""
    ps = _positions(64, 23)
    rng = np.random.default_rng(23)
    pos, moves = [], []
    for p in ps:
        legal = O.fast_gen_moves(p)
        for _ in range(2):
            m = int(rng.choice(legal)) if (len(legal) and rng.random() < 0.7) else int(rng.integers(0, 4096))
            pos.append(pos_of(p))
            moves.append(m)
    pos = np.array(pos, dchess.POS_DTYPE)
    moves = np.array(moves, np.uint16)
    for lo in range(0, len(moves), 64):
        a = live.apply_batch(pos[lo:lo + 64], moves[lo:lo + 64])
        b = engine.apply_batch(pos[lo:lo + 64], moves[lo:lo + 64])
        for x, y in zip(a, b):
            assert (x == y).all()


def test_live_fide_matches_launched(live, engine):
    """FIDE (castling, en passant, promotion) through the mailbox: verdicts and
    made positions equal the launched k_validate_fide / k_apply_fide."""
    ps = _fide_positions(24, 53)
    pos, moves = [], []
    for p in ps:
        legal = [int(m) for m in O.fast_gen_moves(p, O.FIDE)]
        for m in legal[:6] + [legal[0] ^ (1 << 12) if legal else 0, 0x8000, 0x0FFF]:
            pos.append(dpos(p))
            moves.append(m)
    pos = np.array(pos, dchess.POS_DTYPE)
    moves = np.array(moves, np.uint16)
    for lo in range(0, len(moves), 37):
        sl = slice(lo, lo + 37)
        assert (live.validate_batch(pos[sl], moves[sl], rules=FIDE) ==
                engine.validate_batch(pos[sl], moves[sl], rules=FIDE)).all()
        a = live.apply_batch(pos[sl], moves[sl], rules=FIDE)
        b = engine.apply_batch(pos[sl], moves[sl], rules=FIDE)
        for x, y in zip(a, b):
            assert (x == y).all()


def test_live_lease_expiry_and_restart():
    """A short lease: the wave leaves between calls and the next call restarts
    it (the request is taken by exactly one wave); switching the lease off and
    on again keeps every verdict right."""
    pool_pos, pool_mv, pool_want = _pool(24)
    rng = np.random.default_rng(24)
    e = dchess.Engine(0)
    try:
        e.live_validator(2_000)  # 2 ms
        for k in range(12):
            idx = rng.choice(len(pool_mv), 1 + (k % 3) * 20, replace=False)
            assert (e.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all()
            if k % 2:
                time.sleep(0.01)  # past the lease: the wave has left
        e.live_validator(0)
        idx = rng.choice(len(pool_mv), 5, replace=False)
        assert (e.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all()
        e.live_validator(50_000)
        idx = rng.choice(len(pool_mv), 7, replace=False)
        assert (e.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all()
    finally:
        e.live_validator(0)
        e.close()


def test_live_stamp_wrap(live):
    """70,000 requests: the 16-bit stamps wrap (65,535 values) and the request
    area is cleared every 16,384 requests; wide (n = 64) requests are mixed in so
    a stale word of an earlier wide request would be caught."""
    pool_pos, pool_mv, pool_want = _pool(25)
    rng = np.random.default_rng(25)
    idx1 = rng.integers(0, len(pool_mv), 70_000)
    for k in range(70_000):
        if k % 997 == 0:
            idx = rng.choice(len(pool_mv), 64, replace=False)
            assert (live.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all(), k
        i = idx1[k:k + 1]
        assert live.validate_batch(pool_pos[i], pool_mv[i])[0] == pool_want[i[0]], k
