"""GPU check of the FIDE final stage's two split passes (k_count2b<FideRules>,
dc_perft.hip; dc_fide_rules.h fide_count_split / fide_for_each_split).

The kernel sizes each parent's child slots with fide_count_split (visits and
simple children, set-wise) and fills them with fide_for_each_split; if the two
disagreed, slots would overlap or leave gaps with no error raised.  The probe
(tests/kern/split_probe.hip, test-only) runs both passes and fide_for_each_move
on the device for random descendants of startpos and of the published suite
positions, and this test requires:
  - count_split's (visits, ns) == for_each_split's (visits, return value);
  - visits + ns == the number of legal moves (fide_for_each_move, and the oracle);
  - the enumerated moves are the legal moves minus the simple moves of
    tools/fide_simple_proto.py (the set-wise restatement the CPU identity tests
    check against the oracle), in fide_for_each_move's order."""
import ctypes as C
import json
import os
import random
import sys

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tools"))
import fide_simple_proto as F  # noqa: E402

LIB = os.path.join(HERE, "kern", "libsplitprobe.so")
PROBE = np.dtype([("count_c", "<u4"), ("ns_c", "<u4"), ("count_e", "<u4"), ("ns_e", "<u4"), ("n_all", "<u4"),
                  ("pad", "<u4", (3,))])


def positions(n, seed):
    og = json.load(open(os.path.join(HERE, "golden", "oracle_golden.json")))
    roots = [O.Pos()] + [O.Pos.from_fen(e["fen"]) for e in og["perft_fide"].values()]
    rng = random.Random(seed)
    out = []
    for i in range(n):
        pos = roots[i % len(roots)].copy()
        for _ in range(rng.randrange(0, 14) if i % len(roots) else 5):
            mv = O.fast_gen_moves(pos, O.FIDE)
            if len(mv) == 0:
                break
            pos = O.fast_make(pos, int(mv[rng.randrange(len(mv))]), O.FIDE)
        out.append(pos)
    return out


def meta_of(p):
    return p.castle | ((0x400 | (p.ep << 4)) if p.ep >= 0 else 0)


@pytest.mark.gpu
def test_split_passes_agree_and_match_proto():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build()")
    lib = C.CDLL(LIB)
    ps = positions(1200, seed=21)
    n = len(ps)
    bb = np.stack([O.quad(p.cells) for p in ps]).astype(np.uint64)
    stm = np.array([p.stm for p in ps], np.uint8)
    meta = np.array([meta_of(p) for p in ps], np.uint16)
    out = np.zeros(n, PROBE)
    smv = np.zeros((n, 256), np.uint32)
    amv = np.zeros((n, 256), np.uint32)
    vp = C.c_void_p
    rc = lib.split_probe(bb.ctypes.data_as(vp), stm.ctypes.data_as(vp), meta.ctypes.data_as(vp), C.c_uint32(n),
                         out.ctypes.data_as(vp), smv.ctypes.data_as(vp), amv.ctypes.data_as(vp))
    assert rc == 0
    assert (out["count_c"] == out["count_e"]).all()
    assert (out["ns_c"] == out["ns_e"]).all()
    assert (out["count_e"] + out["ns_e"] == out["n_all"]).all()
    simple_total = 0
    for i, p in enumerate(ps):
        legal = O.fast_gen_moves(p, O.FIDE)
        assert int(out["n_all"][i]) == len(legal), i
        allm = [int(x) for x in amv[i, :out["n_all"][i]]]
        assert sorted(allm) == sorted(int(x) for x in legal), i
        simple = set(F.simple_moves(p, legal, F.sens(p)))
        simple_total += len(simple)
        assert int(out["ns_e"][i]) == len(simple), (i, int(out["ns_e"][i]), len(simple))
        assert [int(x) for x in smv[i, :out["count_e"][i]]] == [m for m in allm if m not in simple], i
    assert simple_total > 0.2 * int(out["n_all"].sum())  # the split has work to save on these positions
