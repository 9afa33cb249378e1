import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgpx.so on the device)")


@pytest.fixture(scope="session")
def engine():
    """One GPEngine for the whole GPU session (gpu tests only)."""
    import torch
    from bayesianoptimizer_amd import GPEngine

    assert torch.cuda.is_available(), "gpu tests need a ROCm device"
    return GPEngine(0)
