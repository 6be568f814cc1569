import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhalo_gpu.so)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))


@pytest.fixture(scope="session")
def corc():
    import corc as C
    C.build()
    return C


@pytest.fixture(scope="session")
def hal():
    """The product library on the GPU (gpu tests only)."""
    from halo_amd import _lib as H
    H.ensure_device()
    return H
