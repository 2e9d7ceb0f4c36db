"""CPU check of the REF final stage's target-side pawn correction (k_count3c,
dc_ref.h ref_pawn_planes / ref_parent_split with DC_C2C_GCORR; restated in
tools/ref_gsplit_proto.py).

A quiet move of the side to move whose source is off the opponent's slider
rays and pawn-sensitive squares and whose target is off the rays leaves the
opponent's count at base + pawn_O(parent) + g(t); the kernel counts such
children in bulk on two weight planes.  Checked here against the oracle on
random descendants of startpos and of the REF d6 golden boards (kingless,
unknown-kind and two-king boards among them); the GPU tests pin the kernel
itself through the REF perft goldens (tests/test_gpu_ref.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import ref_gsplit_proto as R  # noqa: E402


def test_target_side_correction_identity():
    st = R.check(1500, seed=7)
    assert st["mismatches"] == 0, st
    # the source-side extension (pawn/knight/king sources on G; not in the kernel)
    assert st["src_mismatches"] == 0 and st["src_bulk"] > 0, st
    # the correction moves most of round 4's enumerated quiet children into the bulk
    assert st["quiet_special_new"] < 0.5 * st["quiet_special_old"], st
