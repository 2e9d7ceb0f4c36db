"""Full-size replay parity (BASELINE configs[3] / [4]) and the multi-GPU replay
combine, on the GPU through libdchess.so.

The golden (tests/golden/replay_golden.json, make_replay_golden.py) is fastcpu
over every game plus refcpu -- the literal restatement of
/root/reference/core/src/chess.rs -- on two 100k-game samples.  Replay
semantics: commit_block (core/src/consensus/hotstuff.rs:52-56)."""
import hashlib
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "replay_golden.json")))
SEED = 0x5EED20241022


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_replay_10m_bit_exact_vs_golden(engine):
    """The north star's target: all 10M games x 80 plies -- generated on the
    device, replayed by k_replay_ref4 -- give the golden moves, accept bitmap,
    per-game digests and counters bit for bit."""
    g = GOLD["c4"]
    n, plies = g["n_games"], GOLD["n_plies"]
    assert n == 10_000_000
    words = (n + 63) // 64
    d_moves = engine.alloc(n * plies * 2)
    d_bm = engine.alloc(words * plies * 8)
    d_dg = engine.alloc(n * 8)
    try:
        engine.gen_games_device(d_moves, SEED, 0, n, plies, GOLD["noise_per_256"])
        st = engine.replay_device(d_moves, n, plies, d_bm, d_dg)
        assert st == g["stats"]
        assert sha(d_bm.download(np.uint64, words * plies)) == g["bitmap_sha256"]
        assert sha(d_dg.download(np.uint64, n)) == g["digests_sha256"]
        assert sha(d_moves.download(np.uint16, n * plies)) == g["moves_sha256"]
    finally:
        for b in (d_moves, d_bm, d_dg):
            b.free()


def test_replay_shards_reassemble_10m(engine):
    """Three dc_replay_shard_range shards of the 10M batch, replayed separately
    and combined as dchess/dist.py does, give the whole batch's golden."""
    import dchess.dist as D
    g = GOLD["c4"]
    n, plies = g["n_games"], GOLD["n_plies"]
    words = (n + 63) // 64
    whole = np.zeros((plies, words), np.uint64)
    recs = []
    for r in range(3):
        first, cnt = dchess.replay_shard_range(n, r, 3)
        w = (cnt + 63) // 64
        d_moves, d_bm = engine.alloc(cnt * plies * 2), engine.alloc(w * plies * 8)
        engine.gen_games_device(d_moves, SEED, first, cnt, plies, GOLD["noise_per_256"])
        st = engine.replay_device(d_moves, cnt, plies, d_bm, None)
        whole[:, first // 64:first // 64 + w] = d_bm.download(np.uint64, w * plies).reshape(plies, w)
        recs.append([st[k] for k in D.STAT_KEYS])
        d_moves.free()
        d_bm.free()
    assert D.fold_stats(recs) == g["stats"]
    assert sha(whole) == g["bitmap_sha256"]


def test_multi_replay_single_device_rccl():
    """dc_multi_replay over one device (ncclGather path) vs fastcpu, ragged size."""
    n, plies = 100_003, 40
    bm, st = dchess.multi_replay([0], SEED, n, plies, 32)
    mv = O.fast_gen_games(SEED, 0, n, plies, 32)
    fbm, _, fst = O.fast_replay(mv)
    assert (bm == fbm).all()
    assert [st[k] for k in ("validated", "accepted", "rejected", "digest_sum", "digest_xor")] == [int(x) for x in fst]


def test_multi_replay_block_of_golden():
    """dc_multi_replay of the first 10M games == the C4 golden."""
    g = GOLD["c4"]
    bm, st = dchess.multi_replay([0], SEED, g["n_games"], GOLD["n_plies"], GOLD["noise_per_256"])
    assert st == g["stats"]
    assert sha(bm) == g["bitmap_sha256"]


@pytest.mark.parametrize("world", [1, 8])
def test_replay_100m_c5_shards_vs_golden(engine, world):
    """BASELINE configs[4]'s 100M-game batch as `world` replay shards (the
    bench's rank layout at N = world, replayed here one shard after another on
    one device), reassembled as dchess/dist.py does: whole-batch bitmap SHA-256
    and combined counters == the C5 golden."""
    import dchess.dist as D
    g = GOLD["c5"]
    n, plies = g["n_games"], GOLD["n_plies"]
    words = (n + 63) // 64
    whole = np.zeros((plies, words), np.uint64)
    recs = []
    for r in range(world):
        first, cnt = D.replay_range(n, r, world)
        w = (cnt + 63) // 64
        d_moves, d_bm = engine.alloc(cnt * plies * 2), engine.alloc(w * plies * 8)
        try:
            engine.gen_games_device(d_moves, SEED, first, cnt, plies, GOLD["noise_per_256"])
            st = engine.replay_device(d_moves, cnt, plies, d_bm, None)
            whole[:, first // 64:first // 64 + w] = d_bm.download(np.uint64, w * plies).reshape(plies, w)
        finally:
            d_moves.free()
            d_bm.free()
        recs.append([st[k] for k in D.STAT_KEYS])
    assert D.fold_stats(recs) == g["stats"]
    assert sha(whole) == g["bitmap_sha256"]
