"""Shared test setup.  `gpu` tests need an MI355X (run with -m gpu on the GPU
box); everything else runs on CPU."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle


def gpu_available() -> bool:
    try:
        import ctypes

        lib = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return lib.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False
