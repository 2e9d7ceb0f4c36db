"""CPU check of the FIDE final stage's simple-child identity (k_count2b
<FideRules> with kSplit, dc_fide_rules.h fide_sens / fide_for_each_split;
restated set-wise in tools/fide_simple_proto.py).

A legal move of the side to move that is quiet and touches none of the
sensitivity sets leaves the opponent's legal move count equal to its count in
the parent with the opponent to move and no en-passant square; the kernel adds
that count for each such child instead of making it.  Checked here against the
oracle (fastcpu) on random descendants of startpos and of the published suite
positions; the GPU tests pin the kernel itself through the published perft
tables (tests/test_gpu_fide.py)."""
import json
import os
import sys

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import fide_simple_proto as F  # noqa: E402

OG = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_golden.json")))


def test_simple_children_startpos_ply5():
    r = F.check([O.Pos()], 1000, seed=11, dmin=5, dmax=5)
    assert r["mismatches"] == 0, r
    assert r["simple_frac"] > 0.3, r  # the split has work to save at perft(7)'s last-but-one ply


def test_simple_children_suite():
    roots = [O.Pos.from_fen(e["fen"]) for e in OG["perft_fide"].values()]
    r = F.check(roots, 1500, seed=12, dmin=0, dmax=14)
    assert r["mismatches"] == 0, r
    assert r["simple"] > 0, r
