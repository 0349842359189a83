"""Shared pytest setup: paths, the `gpu` marker, oracle/libdrhip fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-ranges_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def dr():
    """libdrhip initialised with ONE segment on device 0 (GPU tests only).

    There is deliberately no CPU fallback: a missing library or device
    fails the test instead of skipping it."""
    import drhip
    drhip.load()
    if drhip.device_count() < 1:
        pytest.fail("no HIP device visible for a gpu-marked test")
    drhip.init([0])
    yield drhip
    drhip.finalize()
