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


def test_live_waves_do_not_block_buffer_growth():
    """hipFree / hipHostFree wait for every stream of the device, a resident
    wave's too.  With a 20 s lease on this context and on a second
    one, a perft that grows this context's buffers, a perft on the other
    context, and a context destroyed beside them all finish far inside the
    lease (every resident wave is stopped first, dc_api.hip LiveHold); the
    live calls stay right afterwards."""
    import json
    import os
    og = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
    d5 = og["perft_ref"]["startpos"]["5"]["total"]
    pool_pos, pool_mv, pool_want = _pool(26)
    rng = np.random.default_rng(26)
    a, b = dchess.Engine(0), dchess.Engine(0)
    try:
        a.live_validator(20_000_000)
        b.live_validator(20_000_000)
        for e in (a, b):  # both waves resident
            idx = rng.choice(len(pool_mv), 3, replace=False)
            assert (e.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all()
        steps = {}

        def timed(name, f):
            t0 = time.time()
            r = f()
            steps[name] = round(time.time() - t0, 3)
            return r
        assert timed("perft_a", lambda: a.perft(dchess.startpos(), 5))[0] == d5  # a's buffers grow
        assert timed("perft_b", lambda: b.perft(dchess.startpos(), 5))[0] == d5
        c = timed("create_c", lambda: dchess.Engine(0))
        timed("perft_c", lambda: c.perft(dchess.startpos(), 3))
        timed("close_c", c.close)
        assert sum(steps.values()) < 5.0, steps
        for e in (a, b, a):
            idx = rng.choice(len(pool_mv), 9, replace=False)
            assert (e.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all()
    finally:
        a.live_validator(0)
        b.live_validator(0)
        a.close()
        b.close()


def test_live_timeout_path_then_fresh_verdicts():
    """A call whose answer does not come within the timeout returns DC_EHIP;
    its request is cleared and its stamp burnt, so the next call is never
    answered with the timed-out request's verdict.  The timeout is
    shortened through the test hook dc_test_live_timeout."""
    import ctypes as C
    L = dchess.lib()
    L.dc_test_live_timeout.argtypes = [C.c_void_p, C.c_uint32]
    pool_pos, pool_mv, pool_want = _pool(27)
    ok = np.nonzero(pool_want == 0)[0]
    bad = np.nonzero(pool_want == 3)[0]
    e = dchess.Engine(0)
    try:
        e.live_validator(200_000)
        timeouts = 0
        for k in range(200):
            L.dc_test_live_timeout(e.ctx, 0)
            i = ok[k % len(ok):k % len(ok) + 1]
            out = np.zeros(1, np.uint8)
            pp = np.ascontiguousarray(pool_pos[i])
            mv = np.ascontiguousarray(pool_mv[i])
            r = L.dc_validate_batch(e.ctx, 0, pp.ctypes.data, mv.ctypes.data, 1, out.ctypes.data)
            L.dc_test_live_timeout(e.ctx, 5_000_000)
            if r != 0:
                timeouts += 1
                j = bad[k % len(bad):k % len(bad) + 1]  # a verdict the timed-out request cannot give
                assert e.validate_batch(pool_pos[j], pool_mv[j])[0] == 3
                assert e.validate_batch(pool_pos[i], pool_mv[i])[0] == 0
            else:
                assert out[0] == 0
        assert timeouts > 0
    finally:
        e.live_validator(0)
        e.close()


def test_live_calls_beside_device_work_on_another_thread():
    """a LiveHold on one thread (buffer growth, perft) and live
    calls on another context in a second thread.  live_call decides under
    g_live_mu whether a hold is active (dc_api.hip), so no wave is started
    after a hold has stopped them: every step of the working thread finishes
    far inside the 20 s lease, and every live verdict stays exact."""
    import json
    import os
    import threading
    og = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
    want_perft = {d: og["perft_ref"]["startpos"][str(d)]["total"] for d in (3, 4, 5, 6)}
    pool_pos, pool_mv, pool_want = _pool(27)
    a, b = dchess.Engine(0), dchess.Engine(0)
    stop = threading.Event()
    bad, calls = [], [0]

    def live_loop():
        rng = np.random.default_rng(27)
        while not stop.is_set():
            idx = rng.choice(len(pool_mv), 1 + int(rng.integers(0, 8)), replace=False)
            got = a.validate_batch(pool_pos[idx], pool_mv[idx])
            if not (got == pool_want[idx]).all():
                bad.append(idx)
            calls[0] += 1

    try:
        a.live_validator(20_000_000)
        th = threading.Thread(target=live_loop, daemon=True)
        th.start()
        steps = {}
        for rep in range(3):
            for d in (3, 4, 5, 6):
                t0 = time.time()
                assert b.perft(dchess.startpos(), d)[0] == want_perft[d]
                steps[f"perft{d}_{rep}"] = time.time() - t0
            t0 = time.time()
            mv = b.gen_games(0x5EED + rep, 0, 4096 << rep, 16, 32)  # growing buffers on b
            b.replay(mv)
            steps[f"grow_{rep}"] = time.time() - t0
        stop.set()
        th.join(10)
        assert not th.is_alive()
        assert max(steps.values()) < 5.0, steps
        assert not bad and calls[0] > 0, (len(bad), calls[0])
    finally:
        stop.set()
        a.live_validator(0)
        a.close()
        b.close()
