"""dc_replay_scatter_shards (host, CPU test): the layout dc_multi_replay uses
to put the gathered shard bitmaps back into the whole batch's bitmap, checked
against the shard contract (dc_replay_shard_range, include/dchess.h) and
against dchess/dist.py's combine_replay placement, for uneven shards -- the
case a one-device run never exercises."""
import ctypes as C

import numpy as np
import pytest

import dchess
from dchess import dist as D


def padded_gather(whole, n_games, n_shards):
    """Each shard's word-column block of `whole`, padded to `per` words per row
    (what ncclGather / dist.gather collect), stacked [n_shards][plies][per]."""
    plies, words = whole.shape
    per = (words + n_shards - 1) // n_shards
    out = np.zeros((n_shards, plies, per), np.uint64)
    for i in range(n_shards):
        first, cnt = D.replay_range(n_games, i, n_shards)
        w = (cnt + 63) // 64
        out[i, :, :w] = whole[:, first // 64:first // 64 + w]
    return out


@pytest.mark.parametrize("n_games,n_shards,plies", [(1000, 3, 7), (64 * 5 + 1, 4, 3), (10, 3, 2), (128, 8, 5),
                                                    (100_003, 8, 4), (64, 1, 1)])
def test_scatter_reassembles_whole_bitmap(n_games, n_shards, plies):
    rng = np.random.default_rng(n_games + n_shards)
    words = (n_games + 63) // 64
    whole = rng.integers(0, 2**63, size=(plies, words), dtype=np.uint64)
    if n_games % 64:  # bits past the last game are never set by a replay
        whole[:, -1] &= np.uint64((1 << (n_games % 64)) - 1)
    g = padded_gather(whole, n_games, n_shards)
    # the ABI's range agrees with dist.replay_range (the contract both implement)
    for i in range(n_shards):
        f, c = C.c_uint64(), C.c_uint64()
        assert dchess.lib().dc_replay_shard_range(n_games, i, n_shards, C.byref(f), C.byref(c)) == 0
        assert (f.value, c.value) == D.replay_range(n_games, i, n_shards)
    out = np.zeros((plies, words), np.uint64)
    gc = np.ascontiguousarray(g)
    assert dchess.lib().dc_replay_scatter_shards(n_games, n_shards, plies, gc.ctypes.data, out.ctypes.data) == 0
    assert np.array_equal(out, whole)
    # dist.combine_replay's rank-0 placement loop on the same gathered blocks
    ref = np.zeros((plies, words), np.uint64)
    for r in range(n_shards):
        first, count = D.replay_range(n_games, r, n_shards)
        w = (count + 63) // 64
        ref[:, first // 64:first // 64 + w] = g[r][:, :w]
    assert np.array_equal(ref, whole)


def test_scatter_rejects_bad_arguments():
    out = np.zeros(4, np.uint64)
    assert dchess.lib().dc_replay_scatter_shards(100, 0, 1, out.ctypes.data, out.ctypes.data) == dchess.EINVAL
    assert dchess.lib().dc_replay_scatter_shards(100, 2, 1, None, out.ctypes.data) == dchess.EINVAL
