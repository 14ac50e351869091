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
    """The C ABI with a gfx950 device selected (GPU tests only).

    The parity tests exercise the GPU kernels: the session runs with the SHA-256 host
    offload off and the streaming CRC (piece streams, crc32_update) placed on the GPU
    engine, where the product's defaults (planner-gated offload, the CRC crossover) would
    keep some of these small batches on host threads.  The defaults themselves are tested in
    fresh processes with no knobs set (tests/test_gpu_defaults.py)."""
    from kraken_amd import _capi, device
    n = device.device_count()
    assert n > 0, "no gfx950 device visible (gpu-marked test)"
    device.set_device(0)
    _capi.check(_capi.lib.krk_set_sha_host_offload(0))
    _capi.check(_capi.lib.krk_set_crc_placement(_capi.KRK_PLACE_GPU))
    return device


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(autouse=True)
def _gpu_session_settings(request):
    """Every gpu-marked test runs under the gpu fixture's settings, whichever fixtures it
    names itself."""
    if request.node.get_closest_marker("gpu"):
        request.getfixturevalue("gpu")


def diag_lib() -> str:
    """The diag build of the library (`make diag`: reads the A/B switches of knobs.hpp, which
    the production library does not), built here if missing (build() ships it prebuilt)."""
    import subprocess
    path = os.path.join(ROOT, "kraken_amd", "lib", "diag", "libkraken_hip.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-j", "8", "-C", os.path.join(ROOT, "kraken_amd", "csrc"), "diag"])
    return path
