"""Adversarial co-residency check of the shipped kernels.

A FIDE final-stage variant that is exact when it runs alone (one wave per
SIMD) loses up to half of its leaves when waves of ANOTHER kernel on the same
SIMD issue single-issue VALU instructions (64-bit shifts, v_bcnt, v_add3,
v_cndmask_e64, even VOP2 v_lshlrev_b32), and stays exact beside pairable
VALU, LDS, memory, SALU or sleeping neighbours (tools/diag/noise.hip, round-5
sessions E-J).  This test runs every shipped counting kernel beside exactly
those neighbours -- 512 noise blocks on their own stream, started before and
outlasting the victim -- and requires bit-exact goldens: the REF final stage
k_count3c (perft 6 / 7, and the off-startpos REF d6 positions), the fused
ply-6 words of perft(8), the FIDE final stage k_count2b (suite at depth 5),
and the replay kernel.  The same harness makes the failing variant lose
millions of leaves on every run (profiles/r05/fault_study.md)."""
import ctypes as C
import json
import os
import time

import numpy as np
import pytest

import dchess

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
OG = json.load(open(os.path.join(GOLD, "oracle_golden.json")))
REF_D6 = json.load(open(os.path.join(GOLD, "ref_d6.json")))["positions"]
REF_DEEP = json.load(open(os.path.join(GOLD, "ref_deep.json")))
RG = json.load(open(os.path.join(GOLD, "replay_golden.json")))
KINDS = (1, 6, 12, 13)  # mixed single-issue; 64-bit shifts; v_lshlrev_b32; v_mad_u64_u32


@pytest.fixture(scope="module")
def noise():
    path = os.path.join(REPO, "tools", "diag", "libnoise.so")
    if not os.path.exists(path):
        pytest.fail("tools/diag/libnoise.so not built (__graft_entry__.build())")
    N = C.CDLL(path)
    N.noise_start.argtypes = [C.c_int, C.c_int, C.c_double]

    class Noise:
        def __init__(self, kind, ms):
            self.kind, self.ms = kind, ms

        def __enter__(self):
            assert N.noise_start(self.kind, 512, self.ms) == 0
            time.sleep(0.03)  # the noise blocks are resident before the victim launches
            self.t0 = time.time()

        def __exit__(self, *exc):
            elapsed = time.time() - self.t0
            assert N.noise_wait() == 0
            # the victim must have finished while the noise still ran
            assert elapsed * 1000 < self.ms - 30, f"victim outlasted the noise ({elapsed:.2f} s)"
    return Noise


@pytest.mark.parametrize("kind", KINDS)
def test_ref_final_stage_beside_single_issue_waves(engine, noise, kind):
    s = dchess.startpos()
    for d in (5, 6, 7):
        engine.perft(s, d)  # graphs captured and buffers sized outside the noise window
    got = []
    with noise(kind, 2500):
        for d in (6, 7, 6, 7, 6):
            got.append((d, engine.perft(s, d)[0]))
    for d, t in got:
        assert t == OG["perft_ref"]["startpos"][str(d)]["total"], (kind, d, t)


@pytest.mark.parametrize("kind", (1, 12))
def test_ref_off_startpos_and_perft8_beside_single_issue_waves(engine, noise, kind):
    ps = [(n, dchess.pos_from_cells(np.array(e["cells"], np.int8), e["stm"])) for n, e in sorted(REF_D6.items())]
    for _, p in ps[:1]:
        engine.perft(p, 6)
    engine.perft(dchess.startpos(), 8)
    got = {}
    with noise(kind, 4000):
        for n, p in ps:
            got[n] = engine.perft(p, 6)[0]
        got["startpos_d8"] = engine.perft(dchess.startpos(), 8)[0]
    for n, _ in ps:
        assert got[n] == REF_D6[n]["total"], (kind, n)
    assert got["startpos_d8"] == REF_DEEP["startpos_d8"]["total"]


@pytest.mark.parametrize("kind", KINDS)
def test_fide_final_stage_beside_single_issue_waves(engine, noise, kind):
    names = ["kiwipete", "pos3", "pos4", "pos5", "pos6", "startpos"]
    F = dchess.RULES_FIDE
    for n in names:
        engine.perft(dchess.pos_from_fen(OG["perft_fide"][n]["fen"]), 5, rules=F)
    got = {}
    with noise(kind, 2500):
        for n in names * 2:
            got.setdefault(n, []).append(engine.perft(dchess.pos_from_fen(OG["perft_fide"][n]["fen"]), 5, rules=F)[0])
    for n in names:
        assert got[n] == [OG["perft_fide"][n]["perft"]["5"]] * 2, (kind, n)


@pytest.mark.parametrize("kind", (1, 12))
def test_replay_beside_single_issue_waves(engine, noise, kind):
    """The C4 batch's first 1M games (generated on the device) replayed beside
    the noise: bitmap words and counters equal the undisturbed run's, which the
    10M golden (tests/test_gpu_replay_full.py) pins."""
    mv = engine.gen_games(RG["seed"], 0, 1 << 20, RG["n_plies"], RG["noise_per_256"])
    want = engine.replay(mv)
    with noise(kind, 2500):
        got = [engine.replay(mv) for _ in range(2)]
    for bm, dg, st in got:
        assert (bm == want[0]).all() and (dg == want[1]).all() and st == want[2]


@pytest.mark.parametrize("kind", (1, 12))
def test_fide_validate_replay_beside_single_issue_waves(engine, noise, kind):
    """FIDE kernels outside the final stage that carried the
    compare-overwrite shape until round 6 (tools/vccz_check.py --any) --
    k_validate_fide over every (from, to) pair of suite and game positions,
    k_gen_games_fide + k_replay_fide over 65,536 games -- beside the noise,
    each equal to its undisturbed run (which tests/test_gpu_fide.py pins
    against fastcpu).  The live validator k_live is not stressed here: its
    resident wave and the noise kernels can share one of the process's four
    hardware queues, where one waits for the other instead of co-running (a
    first version of this test timed out that way); the static check covers
    it (tests/test_spill_free.py)."""
    from test_gpu_fide import _fide_positions, dpos
    F = dchess.RULES_FIDE
    ps = _fide_positions(12, 61)
    base = np.array([f | (t << 6) for f in range(64) for t in range(64)], np.uint16)
    pos = np.concatenate([np.repeat(np.array([dpos(p)], dchess.POS_DTYPE), 4096) for p in ps])
    mvs = np.tile(base, len(ps))
    want_v = engine.validate_batch(pos, mvs, rules=F)
    want_g = engine.gen_games(919, 0, 1 << 16, 80, 32, rules=F)
    want_r = engine.replay(want_g, rules=F)
    with noise(kind, 2500):
        got_v = [engine.validate_batch(pos, mvs, rules=F) for _ in range(2)]
        got_g = engine.gen_games(919, 0, 1 << 16, 80, 32, rules=F)
        got_r = engine.replay(got_g, rules=F)
    for g in got_v:
        assert (g == want_v).all()
    assert (got_g == want_g).all()
    assert (got_r[0] == want_r[0]).all() and (got_r[1] == want_r[1]).all() and got_r[2] == want_r[2]
