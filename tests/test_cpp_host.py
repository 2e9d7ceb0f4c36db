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


@pytest.mark.gpu
def test_reference_unit_tests_cpp_host():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout
