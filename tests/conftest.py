import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session")
def gpu():
    """The C ABI with a gfx950 device selected (GPU tests only)."""
    from kraken_amd import device
    n = device.device_count()
    assert n > 0, "no gfx950 device visible (gpu-marked test)"
    device.set_device(0)
    return device


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle
