import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "kolmogorovlike-datacompressor_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_kernels():
    return np.load(os.path.join(GOLDEN, "kernels.npz"))


@pytest.fixture(scope="session")
def golden_containers():
    return np.load(os.path.join(GOLDEN, "containers.npz"))


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def large_known():
    with open(os.path.join(GOLDEN, "large.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kolm_gpu():
    """The product package with its HIP library initialised (GPU tests only)."""
    import kolm
    from kolm import _lib
    _lib.ensure_init()
    return kolm
