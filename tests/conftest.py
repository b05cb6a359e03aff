import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_lib():
    import dvc_amd
    dvc_amd._native.build()
    L = dvc_amd._native.lib()
    import ctypes
    n = ctypes.c_int(0)
    rc = L.dvc_device_count(ctypes.byref(n))
    if rc != 0 or n.value < 1:
        pytest.fail("gpu test without a visible GPU (HIP path has no fallback)")
    return dvc_amd
