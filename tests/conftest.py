import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    oracle_ffi.lib()
    return oracle_ffi


@pytest.fixture(scope="session")
def gpu():
    """The product package with a live device; fails loudly (no fallback) if absent."""
    import lcpc_proof_of_storage_amd as L
    n = L.device_count()
    assert n > 0, "no HIP device visible: the -m gpu tests need an MI355X"
    L.set_device(0)
    return L
