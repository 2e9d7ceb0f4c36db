"""GPU parity tests for RULES_REF: every call goes through libdchess.so (C ABI)
to the gfx950 kernels and is checked bit-exactly against the oracle (refcpu =
literal restatement of core/src/chess.rs; fastcpu = independent engine) and
the committed golden fixtures."""
import hashlib
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KA = json.load(open(os.path.join(GOLD, "known_answers.json")))
OG = json.load(open(os.path.join(GOLD, "oracle_golden.json")))
REF_DEEP = json.load(open(os.path.join(GOLD, "ref_deep.json")))
REF_D6 = json.load(open(os.path.join(GOLD, "ref_d6.json")))["positions"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pos_of(p):
    """oracle Pos -> dc_pos record (via the ABI adapter)."""
    d = dchess.pos_from_cells(p.cells, p.stm)
    d["castle"], d["ep"] = p.castle, p.ep
    return d


# ------------------------------------------------------- reference unit tests
def test_initial_game_state(engine):  # chess.rs:504-514
    g = dchess.GameState("Alice", "Bob", engine)
    assert g.turn == 0 and g.white_player == "Alice" and g.black_player == "Bob"


def test_pawn_valid_move(engine):  # chess.rs:516-530
    g = dchess.GameState("Alice", "Bob", engine)
    g.validate_move(dchess.Position(1, 0), dchess.Position(3, 0))
    g.turn = 1
    g.validate_move(dchess.Position(6, 0), dchess.Position(5, 0))


def test_rook_invalid_move(engine):  # chess.rs:532-539
    g = dchess.GameState("Alice", "Bob", engine)
    with pytest.raises(dchess.AppError):
        g.validate_move(dchess.Position(0, 0), dchess.Position(2, 2))


def test_turn_logic(engine):  # chess.rs:541-556
    g = dchess.GameState("Alice", "Bob", engine)
    g.turn = 0
    g.validate_move(dchess.Position(1, 0), dchess.Position(2, 0))
    g.turn = 1
    g.validate_move(dchess.Position(6, 0), dchess.Position(5, 0))


def test_error_strings_and_panic(engine):
    g = dchess.GameState("Alice", "Bob", engine)
    with pytest.raises(dchess.AppError, match="^No piece at the source location$"):
        g.validate_move(dchess.Position(3, 3), dchess.Position(4, 3))
    with pytest.raises(dchess.AppError, match="^It's not this piece's turn to move$"):
        g.validate_move(dchess.Position(6, 0), dchess.Position(5, 0))
    with pytest.raises(dchess.AppError, match="^Invalid move for the piece$"):
        g.validate_move(dchess.Position(0, 2), dchess.Position(2, 4))
    with pytest.raises(IndexError):
        g.validate_move(dchess.Position(8, 0), dchess.Position(0, 0))


def test_apply_history_sequence(engine):
    seq = KA["apply_sequence"]
    g = dchess.GameState("Alice", "Bob", engine)
    for (f, t) in seq["moves"]:
        g.apply_move(dchess.Position(*f), dchess.Position(*t))
    assert g.history == seq["history"] and g.turn == seq["turn"]
    assert g.board[3][2] == dchess.Piece(0, "B") and g.board[0][5] is None


def test_known_answers_batch(engine):
    s = dchess.startpos()
    pos, moves, want = [], [], []
    for c in KA["validate"]:
        p = s.copy()
        p["stm"] = c["turn"]
        pos.append(p)
        moves.append(dchess.move_pack(*c["from"], *c["to"]))
        want.append(c["verdict"])
    got = engine.validate_batch(np.array(pos, dchess.POS_DTYPE), np.array(moves, np.uint16))
    assert got.tolist() == want


# ------------------------------------------------- exhaustive (from,to) parity
def _positions(n, seed):
    mv = O.fast_gen_games(seed, 0, n, 90, noise_per_256=0)
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n):
        p = O.Pos()
        for ply in range(int(rng.integers(0, 90))):
            m = int(mv[ply, g])
            if m == O.SENTINEL:
                break
            if O.fast_validate(p, m) == O.OK:
                p = O.fast_make(p, m)
        out.append(p)
    return out


@pytest.mark.parametrize("seed", [11, 12])
def test_validate_all_pairs_vs_refcpu(engine, seed):
    ps = _positions(16, seed)
    pos, moves, want = [], [], []
    all_moves = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    for p in ps:
        for stm in (0, 1):
            q = p.copy()
            q.stm = stm
            d = pos_of(q)
            pos.append(np.repeat(np.array([d], dchess.POS_DTYPE), 4096))
            moves.append(all_moves)
            want.append(O.ref_verdicts_all(q.cells, stm))
    got = engine.validate_batch(np.concatenate(pos), np.concatenate(moves))
    assert (got == np.concatenate(want)).all()


def test_validate_odd_pieces_and_oor(engine):
    rng = np.random.default_rng(5)
    pos, moves, want = [], [], []
    all_moves = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    for _ in range(6):
        cells = np.full(64, -1, np.int8)
        sq = rng.choice(64, 24, replace=False)
        cells[sq] = rng.integers(0, 2, 24) * 8 + rng.integers(0, 7, 24)
        for stm in (0, 1):
            pos.append(np.repeat(np.array([dchess.pos_from_cells(cells, stm)], dchess.POS_DTYPE), 4096 + 2))
            moves.append(np.concatenate([all_moves, np.array([dchess.MOVE_OOR, 0x8000 | 77], np.uint16)]))
            want.append(np.concatenate([O.ref_verdicts_all(cells, stm), np.array([4, 4], np.uint8)]))
    got = engine.validate_batch(np.concatenate(pos), np.concatenate(moves))
    assert (got == np.concatenate(want)).all()


def test_validate_batch_sizes_across_paths(engine):
    """Batch sizes either side of the pinned in-place path (<= 4096) and of its
    host completion flag (<= 256), called back to back so every flag value is
    fresh: verdicts equal the literal restatement's, and apply agrees."""
    rng = np.random.default_rng(21)
    ps = _positions(8, 21)
    all_moves = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    pool_pos, pool_want = [], []
    for p in ps:
        for stm in (0, 1):
            q = p.copy()
            q.stm = stm
            pool_pos.append(np.repeat(np.array([pos_of(q)], dchess.POS_DTYPE), 4096))
            pool_want.append(O.ref_verdicts_all(q.cells, stm))
    pool_pos = np.concatenate(pool_pos)
    pool_mv = np.tile(all_moves, len(pool_want))
    pool_want = np.concatenate(pool_want)
    for n in (1, 2, 255, 256, 257, 1, 4096, 4097, 1, 9000, 256, 1):
        idx = rng.choice(len(pool_mv), n, replace=False)
        assert (engine.validate_batch(pool_pos[idx], pool_mv[idx]) == pool_want[idx]).all(), n
        newpos, v, _ = engine.apply_batch(pool_pos[idx], pool_mv[idx])
        assert (v == pool_want[idx]).all(), n
        moved = v == 0  # accepted moves flip the side to move; rejected ones leave the position
        assert (newpos["stm"][moved] != pool_pos[idx]["stm"][moved]).all()
        assert (newpos[~moved] == pool_pos[idx][~moved]).all()


def test_validate_empty_batch(engine):
    assert engine.validate_batch(np.zeros(0, dchess.POS_DTYPE), np.zeros(0, np.uint16)).size == 0


def test_apply_batch_vs_oracle(engine):
    ps = _positions(64, 21)
    pos, moves, exp_pos, exp_v = [], [], [], []
    rng = np.random.default_rng(21)
    for p in ps:
        legal = O.fast_gen_moves(p)
        for _ in range(4):
            m = int(rng.choice(legal)) if (len(legal) and rng.random() < 0.7) else int(rng.integers(0, 4096))
            v = O.fast_validate(p, m)
            q = O.fast_make(p, m) if v == O.OK else p
            pos.append(pos_of(p))
            moves.append(m)
            exp_v.append(v)
            exp_pos.append(pos_of(q))
    new, ver, info = engine.apply_batch(np.array(pos, dchess.POS_DTYPE), np.array(moves, np.uint16))
    assert ver.tolist() == exp_v
    exp = np.array(exp_pos, dchess.POS_DTYPE)
    assert (new["bb"] == exp["bb"]).all() and (new["stm"] == exp["stm"]).all()
    for i, m in enumerate(moves):
        if exp_v[i] == 0:
            cells, _ = dchess.pos_to_cells(pos[i])
            f, t = m & 63, (m >> 6) & 63
            assert info[i] == (cells[f] & 7) | (8 if cells[t] >= 0 else 0)


# ------------------------------------------------------------ generator/replay
def test_gen_games_matches_golden(engine):
    g = OG["games"]
    mv = engine.gen_games(g["seed"], g["first_game"], g["n_games"], g["n_plies"], g["noise_per_256"])
    assert mv[:, 0].tolist() == g["first_game_moves"]
    assert sha(mv) == g["moves_sha256"]
    g2 = OG["games_noise"]
    mv2 = engine.gen_games(g2["seed"], g2["first_game"], g2["n_games"], g2["n_plies"], g2["noise_per_256"])
    assert sha(mv2) == g2["moves_sha256"]


def test_replay_matches_golden(engine):
    for key in ("games", "games_noise"):
        g = OG[key]
        mv = O.fast_gen_games(g["seed"], g["first_game"], g["n_games"], g["n_plies"], g["noise_per_256"])
        bm, dg, st = engine.replay(mv)
        assert sha(bm) == g["bitmap_sha256"] and sha(dg) == g["digests_sha256"]
        assert st == g["stats"]


@pytest.mark.parametrize("n_games,n_plies,noise", [(1, 1, 0), (63, 7, 32), (65, 81, 32), (1000, 80, 255), (4096, 3, 0)])
def test_replay_ragged_vs_fastcpu(engine, n_games, n_plies, noise):
    mv = O.fast_gen_games(7 + n_games, 3, n_games, n_plies, noise_per_256=noise)
    bm, dg, st = engine.replay(mv)
    fbm, fdg, fst = O.fast_replay(mv)
    assert (bm == fbm).all() and (dg == fdg).all()
    assert [st[k] for k in ("validated", "accepted", "rejected", "digest_sum", "digest_xor")] == [int(x) for x in fst]


def test_replay_edge_cases(engine):
    # no plies, sentinel-only games, out-of-range flagged moves, random junk words
    bm, dg, st = engine.replay(np.zeros((0, 10), np.uint16))
    assert st["validated"] == 0 and (dg == O.digest(O.startpos_cells(), 0)).all()
    mv = np.full((5, 70), dchess.MOVE_NONE, np.uint16)
    mv[2, ::3] = dchess.MOVE_OOR
    mv[3, 1::2] = np.random.default_rng(1).integers(0, 0x7FFF, 35)
    bm, dg, st = engine.replay(mv)
    fbm, fdg, fst = O.fast_replay(mv)
    assert (bm == fbm).all() and (dg == fdg).all() and st["validated"] == int(fst[0])


def _replay_from(start, n_games, n_plies, seed):
    """Seeded games from `start` and their expected replay, move by move through
    the literal restatement (refcpu validate_move, chess.rs:82-125; apply as
    chess.rs:72-77).  Mix: legal moves, random 12-bit words, OOR words, and
    games that end early (sentinel rest)."""
    rng = np.random.default_rng(seed)
    mv = np.full((n_plies, n_games), O.SENTINEL, np.uint16)
    bm = np.zeros((n_plies, (n_games + 63) // 64), np.uint64)
    dg = np.zeros(n_games, np.uint64)
    validated = accepted = 0
    for g in range(n_games):
        cells, stm = start.cells.copy(), start.stm
        end = n_plies if rng.random() < 0.8 else int(rng.integers(0, n_plies + 1))
        for ply in range(end):
            r = rng.random()
            legal = O.fast_gen_moves(O.Pos(cells, stm))
            if r < 0.6 and len(legal):
                m = int(rng.choice(legal))
            elif r < 0.95:
                m = int(rng.integers(0, 4096))
            else:
                m = 0x8000 | int(rng.integers(0, 0x7FFF))
            mv[ply, g] = m
            validated += 1
            f, t = m & 63, (m >> 6) & 63
            if m & 0x8000 or O.ref_validate(cells, stm, f >> 3, f & 7, t >> 3, t & 7) != O.OK:
                continue
            cells[t], cells[f] = cells[f], -1
            stm ^= 1
            accepted += 1
            bm[ply, g >> 6] |= np.uint64(1 << (g & 63))
        dg[g] = O.digest(cells, stm)
    return mv, bm, dg, validated, accepted


@pytest.mark.parametrize("kind", ["midgame_black", "odd_pieces"])
def test_replay_from_custom_start_vs_refcpu(engine, kind):
    """dc_replay with start != NULL (the LDS-mailbox kernel packs it on the host)."""
    if kind == "midgame_black":
        start = _positions(1, 44)[0]
        start.stm = 1
    else:
        rng = np.random.default_rng(9)
        cells = np.full(64, -1, np.int8)
        sq = rng.choice(64, 26, replace=False)
        cells[sq] = rng.integers(0, 2, 26) * 8 + rng.integers(0, 7, 26)  # includes kind 6 (OTHER)
        start = O.Pos(cells, 1, 0, -1)
    mv, bm, dg, validated, accepted = _replay_from(start, 100, 37, 5)
    gbm, gdg, st = engine.replay(mv, start=pos_of(start))
    assert (gbm == bm).all() and (gdg == dg).all()
    assert st["validated"] == validated and st["accepted"] == accepted
    assert st["digest_xor"] == int(np.bitwise_xor.reduce(dg))


def test_replay_vs_refcpu_sample(engine):
    mv = engine.gen_games(0x5EED20241022, 123456, 512, 80, 32)
    bm, dg, st = engine.replay(mv)
    rbm, rdg, rst = O.ref_replay(mv, threads=8)
    assert (bm == rbm).all() and (dg == rdg).all()


def test_replay_device_large_properties(engine):
    """1M games x 80 plies resident on the device: size-independent invariants."""
    n, plies = 1 << 20, 80
    d_moves = engine.alloc(n * plies * 2)
    words = (n + 63) // 64
    d_bm = engine.alloc(words * plies * 8)
    d_dg = engine.alloc(n * 8)
    engine.gen_games_device(d_moves, 0x5EED20241022, 0, n, plies, 32)
    st = engine.replay_device(d_moves, n, plies, d_bm, d_dg)
    bm = d_bm.download(np.uint64, words * plies)
    dg = d_dg.download(np.uint64, n)
    mv = d_moves.download(np.uint16, n * plies).reshape(plies, n)
    assert st["validated"] == int((mv != dchess.MOVE_NONE).sum())
    assert st["accepted"] == int(np.unpackbits(bm.view(np.uint8)).sum())
    assert st["accepted"] + st["rejected"] == st["validated"]
    assert st["digest_sum"] == int(dg.sum(dtype=np.uint64))
    assert st["digest_xor"] == int(np.bitwise_xor.reduce(dg))
    # spot-check a sample of games against the oracle
    idx = np.arange(0, n, n // 256)
    sub = np.ascontiguousarray(mv[:, idx])
    _, fdg, _ = O.fast_replay(sub)
    assert (fdg == dg[idx]).all()


# ---------------------------------------------------------------------- perft
@pytest.mark.parametrize("depth", [0, 1, 2, 3, 4, 5, 6, 7])
def test_perft_startpos_golden(engine, depth):
    tot, div, rm = engine.perft(dchess.startpos(), depth)
    if depth == 0:
        assert tot == 1
        return
    g = OG["perft_ref"]["startpos"][str(depth)]
    assert tot == g["total"]
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]


def test_perft_repeated_runs_identical(engine):
    """Repeated perfts of one position (plain runs, then graph replays) all
    equal the golden: the final stage's block-level dynamic scheduling leaves
    no run-to-run variation (round 2 saw a non-shipped LDS-layout variant of
    c2c_group give varying perft(6) counts)."""
    for depth in (5, 6, 7):
        g = OG["perft_ref"]["startpos"][str(depth)]["total"]
        assert [engine.perft(dchess.startpos(), depth)[0] for _ in range(5)] == [g] * 5


def test_perft_random_positions_golden(engine):
    for e in OG["perft_ref"]["random_positions"]:
        d = dchess.pos_from_cells(np.array(e["cells"], np.int8), e["stm"])
        for depth in ("1", "2", "3", "4"):
            assert engine.perft(d, int(depth))[0] == e["perft"][depth]


def test_perft_vs_refcpu_odd_positions(engine):
    rng = np.random.default_rng(9)
    for _ in range(6):
        cells = np.full(64, -1, np.int8)
        sq = rng.choice(64, 18, replace=False)
        cells[sq] = rng.integers(0, 2, 18) * 8 + rng.integers(0, 7, 18)
        for stm in (0, 1):
            want, _ = O.ref_perft(cells, stm, 2, threads=8)
            assert engine.perft(dchess.pos_from_cells(cells, stm), 2)[0] == want
            assert engine.perft(dchess.pos_from_cells(cells, stm), 3)[0] == \
                O.fast_perft(O.Pos(cells, stm, 0, -1), 3)[0]


@pytest.mark.parametrize("n_shards,split", [(2, 1), (3, 2), (8, 3), (5, 4)])
def test_perft_shards_sum(engine, n_shards, split):
    s = dchess.startpos()
    tot, div, rm = engine.perft(s, 5)
    acc = np.zeros_like(div)
    t = 0
    for k in range(n_shards):
        st, sd, srm = engine.perft_shard(s, 5, split, k, n_shards)
        assert (srm == rm).all()
        acc += sd
        t += st
    assert t == tot and (acc == div).all()


@pytest.mark.parametrize("depth,n_shards,split", [(6, 3, 4), (7, 4, 4), (7, 3, 5), (6, 2, 3), (8, 2, 4), (7, 8, 3),
                                                   (6, 8, 3)])
def test_perft_deep_shards_golden(engine, depth, n_shards, split):
    """Strided shards cut after the top kernel (split 3), after k_make_count's
    level (4) or at the final stage's parents (5: k_count2c instead of
    k_count3c), at depths where k_expand_top leaves ply 3 as move words and a
    level write counts the next level: the shards' divides sum to the golden."""
    s = dchess.startpos()
    g = OG["perft_ref"]["startpos"][str(depth)] if depth <= 7 else REF_DEEP["startpos_d8"]
    acc, t = {}, 0
    for k in range(n_shards):
        st, sd, srm = engine.perft_shard(s, depth, split, k, n_shards)
        t += st
        for m, v in zip(srm, sd):
            acc[str(int(m))] = acc.get(str(int(m)), 0) + int(v)
    assert t == g["total"]
    assert acc == {str(k): int(v) for k, v in g["divide"].items()}


@pytest.mark.parametrize("depth,n_shards", [(5, 1), (6, 1), (6, 3), (3, 2)])
def test_perft_repeat_device(engine, depth, n_shards):
    """dc_perft_repeat_device: runs enqueued back to back (graph replays), each
    run's divide / n_root / total left on the device, equal to dc_perft_shard."""
    s = dchess.startpos()
    runs = 3
    W = 258
    for k in range(n_shards):
        st, sd, srm = engine.perft_shard(s, depth, 3 if depth >= 5 else 1, k, n_shards)
        buf = engine.alloc(runs * W * 8)
        engine.perft_repeat_device(s, depth, 3 if depth >= 5 else 1, k, n_shards, runs, buf)
        engine.synchronize()
        res = buf.download(np.uint64, runs * W).reshape(runs, W)
        buf.free()
        for r in res:
            assert int(r[256]) == len(srm)  # n_root, no overflow
            assert int(r[257]) == st
            assert (r[:len(srm)] == sd).all() and not r[len(srm):256].any()
    # a different position after queued runs of the first (the pinned root block changes)
    mid = dchess.pos_from_fen("rnbqkbnr/pppp1ppp/8/4p3/4P3/8/PPPP1PPP/RNBQKBNR w - - 0 2")
    want, _, _ = engine.perft(mid, 4)
    buf = engine.alloc(2 * W * 8)
    engine.perft_repeat_device(s, 4, 1, 0, 1, 1, buf)
    engine.perft_repeat_device(mid, 4, 1, 0, 1, 1, int(buf.ptr.value) + W * 8)
    engine.synchronize()
    res = buf.download(np.uint64, 2 * W).reshape(2, W)
    buf.free()
    assert int(res[0, 257]) == 197742 and int(res[1, 257]) == want


def test_perft_repeat_device_batches(engine):
    """Runs past the batch size go through the 8-run batch graph (captured
    lazily on the first call with >= 8 runs), the rest through the one-run
    graph; every run's result lands at its own slot, also after the root
    position changes between calls."""
    W = 258
    s = dchess.startpos()
    mid = dchess.pos_from_fen("rnbqkbnr/pppp1ppp/8/4p3/4P3/8/PPPP1PPP/RNBQKBNR w - - 0 2")
    want_mid, _, _ = engine.perft(mid, 5)
    want_s = 4896998  # REF perft(5) of startpos (tests/golden)
    for pos, want, runs in ((s, want_s, 2), (s, want_s, 19), (mid, want_mid, 9), (s, want_s, 8)):
        buf = engine.alloc(runs * W * 8)
        engine.perft_repeat_device(pos, 5, 3, 0, 1, runs, buf)
        engine.synchronize()
        res = buf.download(np.uint64, runs * W).reshape(runs, W)
        buf.free()
        assert (res[:, 257] == want).all(), res[:, 257]


def test_perft_repeat_device_split_over_contexts(engine):
    """The bench's timed perft steps split over concurrent contexts (bench.py
    enqueue_split): three contexts -- three streams -- enqueue their shares of
    whole runs at once, each into its slots of ONE result array allocated by
    another context, two of them with a different position; every record is
    the right whole perft."""
    W = 258
    s = dchess.startpos()
    mid = dchess.pos_from_fen("rnbqkbnr/pppp1ppp/8/4p3/4P3/8/PPPP1PPP/RNBQKBNR w - - 0 2")
    want_mid, _, _ = engine.perft(mid, 6)
    want_s = 120909581  # REF perft(6) of startpos (tests/golden)
    others = [dchess.Engine(0), dchess.Engine(0)]
    engs = [engine] + others
    jobs = [(s, want_s, 9), (mid, want_mid, 10), (s, want_s, 11)]
    total = sum(n for _, _, n in jobs)
    buf = engine.alloc(total * W * 8)
    try:
        for e, (p, _, n) in zip(engs, jobs):  # captures first (a plain run per context)
            e.perft_repeat_device(p, 6, 3, 0, 1, 1, buf)
            e.synchronize()
        k0 = 0
        for e, (p, _, n) in zip(engs, jobs):
            e.perft_repeat_device(p, 6, 3, 0, 1, n, int(buf.ptr.value) + k0 * W * 8)
            k0 += n
        for e in engs:
            e.synchronize()
        res = buf.download(np.uint64, total * W).reshape(total, W)
    finally:
        buf.free()
        for e in others:
            e.close()
    want = np.concatenate([np.full(n, w, np.uint64) for _, w, n in jobs])
    assert (res[:, 257] == want).all(), res[:, 257]
    assert not (res[:, 256] >> np.uint64(32)).any()


def test_perft_repeat_device_profiling_then_other_position(engine):
    """With profiling on, dc_perft_repeat_device enqueues plain (non-graph) runs,
    each copying the pinned root block when it executes; a perft of another
    position issued right after must not overwrite that block under them."""
    s = dchess.startpos()
    mid = dchess.pos_from_fen("rnbqkbnr/pppp1ppp/8/4p3/4P3/8/PPPP1PPP/RNBQKBNR w - - 0 2")
    want_mid, _, _ = engine.perft(mid, 5)
    W, runs = 258, 4
    buf = engine.alloc(runs * W * 8)
    engine.set_profiling(True)
    try:
        engine.perft_repeat_device(s, 5, 3, 0, 1, runs, buf)
        got_mid, _, _ = engine.perft(mid, 5)  # host path: writes the pinned root block
        engine.synchronize()
    finally:
        engine.set_profiling(False)
    res = buf.download(np.uint64, runs * W).reshape(runs, W)
    buf.free()
    assert got_mid == want_mid
    assert (res[:, 257] == 4896998).all()


def test_multi_perft_single_device_rccl():
    """dc_multi_perft over one device: RCCL communicator + all-reduce path."""
    s = dchess.startpos()
    tot, div, rm = dchess.multi_perft([0], s, 5)
    g = OG["perft_ref"]["startpos"]["5"]
    assert tot == g["total"]
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]


def test_sharded_perft_combine_single_rank(engine):
    import dchess.dist as D
    s = dchess.startpos()
    tot, div, rm = D.sharded_perft(lambda p, d, sp, r, w: engine.perft_shard(p, d, sp, r, w), s, 6, 3, 0, 1)
    assert tot == OG["perft_ref"]["startpos"]["6"]["total"]


def test_perft_suite_fens_ref_rules(engine):
    """SURVEY §8d C3, REF half: the standard-suite FENs under the reference's
    rules (castling/ep fields carried but ignored) at depth 5."""
    for name, e in OG["perft_ref"]["suite"].items():
        p = dchess.pos_from_fen(e["fen"])
        for d in ("3", "5"):
            assert engine.perft(p, int(d))[0] == e["perft"][d], (name, d)


@pytest.mark.parametrize("name", sorted(REF_D6))
def test_perft6_ref_off_startpos_tree(engine, name):
    """REF perft(6) with divide of the six suite FENs and ten mid-game boards
    (four edited: no white king, no kings, unknown-kind pieces, two white
    kings -- chess.rs:199-212, 350-360), fastcpu-pinned and refcpu-checked on a
    subtree each (tests/golden/make_ref_d6_golden.py).  Their final stage runs
    k_count3c on a full grid (0.3M-9M move words) where the startpos goldens
    were the only full-occupancy pins; then again as 8 strided shards cut after
    the top kernel, whose divides must sum to the same vector."""
    e = REF_D6[name]
    p = dchess.pos_from_cells(np.array(e["cells"], np.int8), e["stm"])
    tot, div, rm = engine.perft(p, 6)
    assert tot == e["total"]
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == e["divide"]
    acc, t = {}, 0
    for k in range(8):
        st, sd, srm = engine.perft_shard(p, 6, 3, k, 8)
        t += st
        for m, v in zip(srm, sd):
            acc[str(int(m))] = acc.get(str(int(m)), 0) + int(v)
    assert t == e["total"]
    assert {m: v for m, v in acc.items() if v} == {m: v for m, v in e["divide"].items() if v}


def test_front_path_taken_and_declined(engine):
    """Round 6's one-launch front end (k_front, dc_perft.hip): REF perft(6) and
    perft(7) of one root, unsharded or a strided shard of ply 3, run it; a
    position whose ply 2 is past its LDS bound (pos6 of ref_d6: 2,124 ply-2
    nodes > 2,048) is declined on the device and rerun on the legacy chain;
    other shapes (split 4, depth 5, FIDE) never take it.  Totals are the
    goldens either way (dc_test_perft_last_front reports the path)."""
    import ctypes as C
    L = dchess.lib()
    L.dc_test_perft_last_front.argtypes = [C.c_void_p]
    front = lambda: L.dc_test_perft_last_front(engine.ctx)  # noqa: E731
    s = dchess.startpos()
    for d in (6, 7):
        for _ in range(2):  # the plain run, then the captured graph
            assert engine.perft(s, d)[0] == OG["perft_ref"]["startpos"][str(d)]["total"]
            assert front() == 1
    t = 0
    for k in range(8):
        t += engine.perft_shard(s, 7, 3, k, 8)[0]
        assert front() == 1
    assert t == OG["perft_ref"]["startpos"]["7"]["total"]
    engine.perft_shard(s, 7, 4, 1, 8)
    assert front() == 0
    assert engine.perft(s, 5)[0] == OG["perft_ref"]["startpos"]["5"]["total"]
    assert front() == 0
    for name, want in (("pos6", 0), ("mid4", 1), ("pos6", 0)):
        e = REF_D6[name]
        p = dchess.pos_from_cells(np.array(e["cells"], np.int8), e["stm"])
        assert engine.perft(p, 6)[0] == e["total"]
        assert front() == want, name


# ------------------------------------------------------------- replicas (C1)
def test_four_replicas_scripted_game():
    """four in-process replicas (one dc_ctx each, as each
    HotStuff peer owns its validator) apply one scripted game with three
    injected illegal moves through the GameState mirror (chess.rs:43-98); all
    must agree with each other and with refcpu on every verdict, the history
    string, the final board and its digest."""
    g = OG["replica_game"]
    reps = [dchess.GameState("Alice", "Bob", dchess.Engine(0)) for _ in range(4)]
    seen = []
    for r in reps:
        vs = []
        for fx, fy, tx, ty in g["moves"]:
            try:
                r.apply_move(dchess.Position(fx, fy), dchess.Position(tx, ty))
                vs.append(0)
            except dchess.AppError as e:
                vs.append({dchess.verdict_message(k): k for k in (1, 2, 3)}[str(e)])
        cells = np.array([-1 if c is None else c.color * 8 + "PNBRQK".index(c.kind)
                          for row in r.board for c in row], np.int8)
        seen.append((vs, r.history, r.turn, cells.tolist()))
    for vs, hist, turn, cells in seen:
        assert vs == g["verdicts"] and hist == g["history"] and turn == g["turn"]
        assert cells == g["final_cells"]
    assert O.digest(np.array(seen[0][3], np.int8), seen[0][2]) == g["final_digest"]
