"""The planners' rates measured on the device (krk_planner_rates_get, offload.cpp
calibrate): each SHA-256 tier's per-stream rate at full residency, pinned copy rates,
one host thread's SHA-256 / CRC-32 rates -- and the offload plan of a device batch
priced with them."""
import pytest

from kraken_amd import device as D

pytestmark = pytest.mark.gpu


def test_rates_measured_on_device(gpu):
    R = D.planner_rates()
    print(R)
    assert R["source"] == "measured"
    s8, s2, s1 = R["sha_stream_bps"]
    # per-stream SHA-256: eight lanes > two lanes > one lane, all tens of MB/s
    assert 30e6 < s1 < s2 < s8 < 120e6, R
    assert 10e9 < R["h2d_bps"] < 80e9 and 10e9 < R["d2h_bps"] < 80e9, R
    assert R["host_sha_bps"] > 1e8 and R["host_crc_bps"] > 1e8
    assert R["cus"] >= 1
    assert D.planner_rates() == R  # measured once per device
    # C1 (one 1 GiB blob): the host thread's chain beats one GPU stream
    assert list(D.sha_offload_plan([1 << 30], 4)[0]) == [0]
    assert D.sha_offload_plan([100 << 20] * 1000, 16)[0].size == 0  # C2 stays on the GPU
