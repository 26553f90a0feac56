"""The driver's smoke check (__graft_entry__.smoke) as a GPU test: hot-path and full
candidate containers against the oracle, decoded back on the device."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_graft_smoke(kolm_gpu):
    sys.path.insert(0, REPO)
    import __graft_entry__
    __graft_entry__.smoke()
