"""K4 -- per-lane DFS perft (k_perft_dfs) -- on the GPU through libdchess.so.

Under RULES_REF a perft deeper than 8 keeps its BFS levels at ply <= 5 and
walks the remaining L = depth - 7 plies above the two-ply final stage per
lane with an explicit stack.  perft(8) takes the fused final
stage below ply 5 with 64-bit move words (k_level_moves + k_count3c) and falls
back to K4 (L = 1) when ply 6 is too large; DCHESS_PERFT_K4=1 forces K4 there,
so both depth-8 paths are checked.  Checked against
  * fastcpu (oracle/fastcpu.cpp) on sparse positions at depths 8, 9 and 10
    (L = 1, 2, 3), computed in the test;
  * the committed startpos perft(8) divide (tests/golden/ref_deep.json,
    make_deep_golden.py), directly, sharded and through repeated device runs.
"""
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

pytestmark = pytest.mark.gpu

DEEP = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_deep.json")))

SPARSE = [
    ("4k3/8/8/8/8/8/8/R3K3 w - - 0 1", 8),       # L = 1
    ("7k/8/8/8/3N4/8/8/K7 b - - 0 1", 8),        # L = 1, black to move at the root
    ("7k/8/8/8/8/8/8/K7 w - - 0 1", 9),          # L = 2
    ("8/8/2k5/8/8/5K2/8/8 b - - 0 1", 9),        # L = 2
    ("k7/8/8/8/8/8/8/7K w - - 0 1", 10),         # L = 3
]


@pytest.fixture(params=["fused", "k4"])
def d8_path(request, monkeypatch):
    """The depth-8 path: the fused final stage below ply 5 (default) or K4."""
    if request.param == "k4":
        monkeypatch.setenv("DCHESS_PERFT_K4", "1")
    else:
        monkeypatch.delenv("DCHESS_PERFT_K4", raising=False)
    return request.param


@pytest.mark.parametrize("fen,depth", SPARSE, ids=[f"d{d}-{i}" for i, (_, d) in enumerate(SPARSE)])
def test_dfs_sparse_vs_fastcpu(engine, fen, depth, d8_path):
    if depth > 9 and d8_path == "fused":
        pytest.skip("the path switch applies at depths 8 and 9 only")
    p = O.Pos.from_fen(fen)
    want, wdiv, wrm = O.fast_perft(p, depth, O.REF, threads=min(16, os.cpu_count() or 1))
    tot, div, rm = engine.perft(dchess.pos_from_fen(fen), depth)
    assert tot == want
    assert dict(zip(rm.tolist(), div.tolist())) == dict(zip(wrm.tolist(), wdiv.tolist()))


def test_perft8_startpos_golden(engine, d8_path):
    g = DEEP["startpos_d8"]
    tot, div, rm = engine.perft(dchess.startpos(), 8)
    assert tot == g["total"]
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]
    assert engine.perft(dchess.startpos(), 8)[0] == g["total"]  # the captured graph's replay
    engine.reset_stats()
    engine.set_profiling(True)
    try:
        assert engine.perft(dchess.startpos(), 8)[0] == g["total"]
        dfs, fin = engine.kernel_stats("dfs")["launches"], engine.kernel_stats("count2")["launches"]
    finally:
        engine.set_profiling(False)
    assert (dfs, fin) == ((1, 0) if d8_path == "k4" else (0, 1))  # the path asked for ran


def test_perft8_wide_overflow_falls_back_to_k4(monkeypatch):
    """A ply 6 larger than the 64-bit word capacity: the speculative run is
    flagged, the exact rerun sees the word count and takes K4 from ply 5
    (capacity lowered through DCHESS_PERFT_WIDE_MAX on a fresh context)."""
    monkeypatch.delenv("DCHESS_PERFT_K4", raising=False)
    monkeypatch.setenv("DCHESS_PERFT_WIDE_MAX", "1000")
    fen = SPARSE[0][0]
    want, _, _ = O.fast_perft(O.Pos.from_fen(fen), 8, O.REF, threads=min(16, os.cpu_count() or 1))
    eng = dchess.Engine(0)
    eng.set_profiling(True)
    assert eng.perft(dchess.pos_from_fen(fen), 8)[0] == want
    assert eng.kernel_stats("dfs")["launches"] == 1


@pytest.mark.parametrize("n_shards", [3, 8])
def test_perft8_shards_sum(engine, n_shards, d8_path):
    s = dchess.startpos()
    acc, t = None, 0
    for k in range(n_shards):
        st, sd, _ = engine.perft_shard(s, 8, 3, k, n_shards)
        acc = sd.copy() if acc is None else acc + sd
        t += st
    assert t == DEEP["startpos_d8"]["total"]


def test_perft8_repeat_device(engine, d8_path):
    s = dchess.startpos()
    W, runs = 258, 2
    buf = engine.alloc(runs * W * 8)
    engine.perft_repeat_device(s, 8, 3, 0, 1, runs, buf)
    engine.synchronize()
    res = buf.download(np.uint64, runs * W).reshape(runs, W)
    buf.free()
    assert (res[:, 257] == DEEP["startpos_d8"]["total"]).all()
    assert not (res[:, 256] >> np.uint64(32)).any()


def test_perft9_startpos_golden(engine, d8_path):
    """perft(startpos, 9): total and divide against fastcpu's golden (2.6e12
    leaves, 2.5 h on 8 host threads) through the sliced fused final stage
    (ply 6 as boards, 4.3 GB; ply 7 as 64-bit words per slice of 2^21 ply-6
    nodes) and through K4 at L = 2 (explicit per-lane stack of one frame, BFS
    levels stopping at ply 5)."""
    g = DEEP["startpos_d9"]
    tot, div, rm = engine.perft(dchess.startpos(), 9)
    assert tot == g["total"] == 2_597_923_551_373
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]


def test_perft9_wide_level_overflow_falls_back_to_k4(monkeypatch):
    """Ply 6 larger than the sliced stage's level budget: the speculative run is
    flagged, the exact rerun takes K4 from ply 5 (budget lowered through
    DCHESS_PERFT_WIDE_LEVEL_MAX on a fresh context, sparse position)."""
    monkeypatch.delenv("DCHESS_PERFT_K4", raising=False)
    monkeypatch.setenv("DCHESS_PERFT_WIDE_LEVEL_MAX", "100000")
    fen = SPARSE[2][0]
    want, _, _ = O.fast_perft(O.Pos.from_fen(fen), 9, O.REF, threads=min(16, os.cpu_count() or 1))
    eng = dchess.Engine(0)
    eng.set_profiling(True)
    assert eng.perft(dchess.pos_from_fen(fen), 9)[0] == want
    assert eng.kernel_stats("dfs")["launches"] == 1


def test_depth_beyond_k4_unsupported(engine):
    with pytest.raises(dchess.DChessError) as e:
        engine.perft(dchess.startpos(), 11)
    assert e.value.status == dchess.EUNSUPPORTED


# ------------------------------------------- refcpu-agreed deep pins (make_deep_golden.py)
def test_startpos_d5_divide_pinned_by_refcpu(engine):
    g = DEEP["startpos_d5"]
    assert g["engines"] == ["refcpu", "fastcpu"]
    tot, div, rm = engine.perft(dchess.startpos(), 5)
    assert tot == g["total"]
    assert {str(int(m)): int(v) for m, v in zip(rm, div)} == g["divide"]


def test_startpos_d6_subtrees_pinned_by_refcpu(engine):
    tot, div, rm = engine.perft(dchess.startpos(), 6)
    got = {str(int(m)): int(v) for m, v in zip(rm, div)}
    for m, v in DEEP["startpos_d6_subtrees"]["divide"].items():
        assert got[m] == v


def test_suite_d4_pinned_by_refcpu(engine):
    for name, e in DEEP["suite_d4"]["positions"].items():
        p = dchess.pos_from_fen(e["fen"])
        for d, v in e["perft"].items():
            assert engine.perft(p, int(d))[0] == v, (name, d)


def test_random_d3_pinned_by_refcpu(engine):
    for e in DEEP["random_d3"]["positions"]:
        p = dchess.pos_from_cells(np.array(e["cells"], np.int8), e["stm"])
        assert engine.perft(p, 3)[0] == e["perft3"]
