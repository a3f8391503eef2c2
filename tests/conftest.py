import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X) and libpfe.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def engine():
    """One libpfe handle on cuda:0 for the whole GPU test session (fails loudly)."""
    from pulsarfeatureextractor_amd._native import Engine

    e = Engine(0)
    yield e
    e.close()
