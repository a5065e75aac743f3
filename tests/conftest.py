import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: large parity sizes")


@pytest.fixture(scope="session")
def gpu_engine_lib():
    """The product library; GPU tests must never fall back to anything else."""
    import corrosion_amd._lib as L
    return L.lib()
