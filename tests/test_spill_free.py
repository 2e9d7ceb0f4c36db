"""The shipped REF kernels use no scratch (CPU test, reads the built library's
gfx950 code objects).  Round 2's only wrong perft counts came from final-stage
builds that spilled registers to scratch at 4 waves/SIMD (DESIGN.md section
7); since round 3 every REF perft, replay and validation kernel is built
spill-free, and this test keeps it so: .private_segment_fixed_size == 0 in the
AMDGPU metadata of every such kernel.  The signature kernel joined them late in
round 3 (its Q table was SGPR-indexed in scratch; now 248 VGPRs, 0 B)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import dchess

LLVM = "/opt/rocm/lib/llvm/bin"
# mangled-name fragments of the kernels that must stay spill-free
MUST = ("k_count3c", "k_count2c", "k_front", "k_perft_dfs", "k_replay_ref4", "k_validate_ref", "k_apply_ref",
        "k_gen_games_ref", "RefRules", "FideRules", "k_verify_tx", "k_live")


def kernel_scratch():
    tmp = tempfile.mkdtemp()
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(dchess.LIB_PATH, lib)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", lib], cwd=tmp, check=True,
                       capture_output=True)
        out = {}
        for f in os.listdir(tmp):
            if not f.endswith("gfx950"):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(tmp, f)],
                                   check=True, capture_output=True, text=True).stdout
            name = None
            for line in notes.splitlines():
                m = re.match(r"\s*\.name:\s+(\S+)", line)
                if m:
                    name = m.group(1)
                m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
                if m and name:
                    out[name] = int(m.group(1))
        return out
    finally:
        shutil.rmtree(tmp)


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-readelf")), reason="no ROCm llvm tools")
def test_ref_kernels_are_spill_free():
    ks = kernel_scratch()
    checked = {n: s for n, s in ks.items() if any(p in n for p in MUST)}
    assert len(checked) >= 20, sorted(ks)
    spilling = {n: s for n, s in checked.items() if s != 0}
    assert not spilling, spilling


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="no ROCm llvm tools")
def test_scratch_bounds_and_lane_spills():
    """tools/scratch_bounds_check.py on every kernel of the built library: no
    scratch access outside its kernel's private segment, none through a VGPR
    or untraced SGPR address, no SGPR-spill VGPR written under a partial EXEC
    (the two mechanisms examined for the round-2 fault,
    and the address-select that kept the FIDE analysis in scratch)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import scratch_bounds_check as sbc
    ks = sbc.kernels_from_lib(dchess.LIB_PATH)
    assert len(ks) >= 40, sorted(ks)
    bad = {}
    for name, (lines, priv, dyn) in ks.items():
        b, lanes, _, _ = sbc.check_kernel(lines, priv, dyn)
        if b or lanes:
            bad[name] = (b + lanes)[:3]
    assert not bad, bad


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="no ROCm llvm tools")
def test_no_kernel_has_the_round5_fault_window():
    """tools/vccz_check.py --any on every kernel of the built library: no VCCZ
    branch whose VALU compare has its source registers overwritten by ANY VALU
    write before the branch -- the window whose preemption by a co-resident
    wave's single-issue VALU instruction made the round-4 table variant lose
    up to half of its leaves (round 5 checked only
    64-bit shift writers, and 16 FIDE kernels still had v_and_b32 writers).
    The FIDE analysis makes the king's half-line masks and all four line-gate
    operands before its gates, each kept live past its branch (dc_fide_rules.h)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import scratch_bounds_check as sbc
    import vccz_check
    ks = sbc.kernels_from_lib(dchess.LIB_PATH)
    assert len(ks) >= 200, len(ks)
    bad = {n: vccz_check.shape(lines, any_writer=True)[:1] for n, (lines, _, _) in ks.items()
           if vccz_check.shape(lines, any_writer=True)}
    assert not bad, bad
