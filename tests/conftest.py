import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def root():
    return ROOT


def cfg_path(*parts):
    return os.path.join(ROOT, "configs", *parts)
