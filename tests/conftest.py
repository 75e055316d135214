import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs through the HIP C ABI")
    config.addinivalue_line("markers", "slow: multi-second CPU work")


@pytest.fixture(scope="session")
def oracle():
    from tests import _support
    return _support.load_oracle()


@pytest.fixture(scope="session")
def lhpc():
    import libhpc_amd
    return libhpc_amd


@pytest.fixture(scope="session")
def gpu(lhpc):
    """Fails loudly (not skips) when a gpu-marked test runs without a device."""
    if lhpc.device_count() < 1:
        pytest.fail("gpu test selected but no gfx950 device is visible")
    import torch
    assert torch.cuda.is_available(), "torch sees no GPU"
    return torch.device("cuda:0")
