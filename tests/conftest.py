import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs through libdchess.so)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle check")


@pytest.fixture(scope="session")
def engine():
    import dchess
    e = dchess.Engine(0)
    yield e
    e.close()
