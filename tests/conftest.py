import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); runs through the C ABI")
    config.addinivalue_line("markers", "slow: long CPU-oracle runs (minutes)")


@pytest.fixture(scope="session")
def raftmc():
    import importlib
    return importlib.import_module("raft-tla_amd")
