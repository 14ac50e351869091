"""The C3 host lane's planner (kraken_amd.windowed.host_lane_plan), host only: how many
of a windowed batch's longest blobs go to host threads, from the planner rates.  The
rates are injected (the GPU box's measured figures: ~58 MB/s an eight-lane stream,
51.6 MB/s two lanes, ~2.1 GB/s a SHA-NI thread, ~54 GB/s D2H) so the answer does not
depend on this container's CPU."""
import numpy as np

from kraken_amd.shard import lpt_shard
from kraken_amd.windowed import c3_lengths, host_lane_plan, window_plan, windows_seconds

BOX = {"sha_stream_bps": [58e6, 51.6e6, 35.7e6], "d2h_bps": 54e9, "h2d_bps": 54e9, "host_sha_bps": 2.1e9,
       "host_crc_bps": 8e9, "host_copy_bps": 10e9, "cus": 256, "source": "set"}
W, CAP = 48 << 30, 14336


class _NoDevice:  # host_lane_plan takes its rates from D only when none are given
    def planner_rates(self):
        raise AssertionError("rates were passed")


def test_emulated_rank_of_eight_takes_hundreds_of_blobs():
    L = c3_lengths(20000)
    shard = [L[i] for i in lpt_shard(L, 8)[0]]
    k, t, t0 = host_lane_plan(_NoDevice(), shard, W, CAP, 15, rates=BOX)
    assert k % 15 == 0 and 300 <= k <= 700
    assert t < 0.88 * t0  # the shard's windows shrink by more than an eighth
    # the chosen K balances the two sides: one group more or less is no better
    order = np.argsort(-np.asarray(shard), kind="stable")
    for kk in (k - 15, k + 15):
        rest = [shard[i] for i in order[kk:]]
        host = sum(shard[order[g]] for g in range(0, kk, 15)) / min(BOX["host_sha_bps"], BOX["d2h_bps"] / 15)
        assert max(windows_seconds(BOX, rest, W, CAP), host) >= t - 1e-9


def test_slow_host_keeps_everything_on_the_gpu():
    L = c3_lengths(2500)
    slow = dict(BOX, host_sha_bps=50e6)  # a host thread no faster than a GPU stream
    assert host_lane_plan(_NoDevice(), L, W, CAP, 15, rates=slow)[0] == 0


def test_windows_model_is_the_sum_of_window_chains():
    L = c3_lengths(300, scale=64)
    wins = window_plan(L, 1 << 30, 100)
    want = sum(float(t.max()) / 58e6 + 0.0005 for _, _, t in wins)
    assert abs(windows_seconds(BOX, L, 1 << 30, 100) - want) < 1e-9


def test_lane_groups_stop_at_k():
    """The lane hashes groups of `threads` of the K longest blobs; a K that is not a multiple
    of `threads` leaves a short last group, never blobs past K (the GPU lane test's 100 = 12 x
    8 + 4 once took the four longest window blobs as well, and their piece sums broke)."""
    from kraken_amd.windowed import lane_groups
    L = c3_lengths(1500, scale=16)
    order = np.argsort(-np.asarray(L), kind="stable")
    for k, t in [(100, 8), (96, 8), (7, 8), (0, 8), (480, 15), (1500, 7), (2000, 7)]:
        blobs, groups = lane_groups(L, k, t)
        kk = min(k, len(L))
        assert sorted(np.concatenate(groups).tolist() if groups else []) == sorted(order[:kk].tolist())
        assert blobs.tolist() == sorted(order[:kk].tolist())
        assert all(len(g) == t for g in groups[:-1]) and (not groups or 1 <= len(groups[-1]) <= t)
        assert len(groups) == -(-kk // t)
