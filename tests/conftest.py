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


@pytest.fixture(autouse=True)
def _reset_gnn_cu_budget():
    """A trainer in overlap mode sets the native module's process-wide GNN CU budget (work-queue grids, whose
    gradient summation order follows the claim order); a test that ran one before must not leave later tests --
    the bitwise-determinism checks -- in that mode."""
    nat = sys.modules.get("gsc_amd._native")
    if nat is not None:
        nat.gnn_set_cu_budget(0)
    yield
