"""The reference's own unit tests (core/src/chess.rs:499-557), restated in C++
against the host mirror (distributed-chess_amd/host/chess_state.hpp) and run
through the C ABI on the GPU."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "distributed-chess_amd", "build", "test_chess_rs")


def test_cpp_binary_built():
    assert os.path.exists(EXE), "run __graft_entry__.build()"


def test_cpp_host_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "no usable gfx950 device" in r.stdout


def test_cpp_state_json_and_hash_vs_oracle():
    """GameState::to_json / state_hash of the C++ mirror (host only) against the
    oracle's serde_json restatement + keccak256 (oracle/statehash.py)."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import statehash as S
    r = subprocess.run([EXE, "--json"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    cells = np.full(64, -1, np.int8)
    for y, k in enumerate([3, 1, 2, 4, 5, 2, 1, 3]):  # RNBQKBNR in dchess.h cell kind codes
        cells[y], cells[56 + y] = k, 8 + k
    cells[8:16], cells[48:56] = 0, 8
    cells[28], cells[12] = 0, -1      # e2 -> e4
    cells[36], cells[52] = 8, -1      # e7 -> e5
    cells[45] = 8 + 6                 # a kind string outside P N B R Q K
    names = ("Al\"ice\\", "B\tob\x01")
    for i, (turn, hist) in enumerate([(0, "1. e4 3. e5"), (1, None)]):
        want = S.game_state_json(turn, *names, hist, cells, kinds={45: "Dragon"})
        assert lines[2 * i] == want
        assert lines[2 * i + 1] == S.state_hash(turn, *names, hist, cells, kinds={45: "Dragon"})


@pytest.mark.gpu
def test_reference_unit_tests_cpp_host():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout
