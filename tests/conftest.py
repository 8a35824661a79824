import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "insr-pde_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_sessionstart(session):
    """INSR_TEST_BWD_F16=<mask>: run the suite with that INSR_JET_BWD_F16 mask in every jet call of
    the test thread (A/B of a default before it is made one; test infrastructure only)."""
    mask = os.environ.get("INSR_TEST_BWD_F16")
    if mask is not None:
        import base
        base._native.set_default_knobs(bwd_f16=int(mask))
