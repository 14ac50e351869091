"""The C3 host lane's rate, alone and beside the GPU windows (kraken_amd.windowed).
KRK_TRACE=1 adds one stderr line per lane group: wall, and per-thread sums of the time
spent waiting for the D2H copies and hashing.

    python tools/lane_probe.py [--k 60] [--threads 15] [--mode alone|windows|both]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kraken_amd import device as D  # noqa: E402
from kraken_amd.shard import lpt_shard  # noqa: E402
from kraken_amd.windowed import WindowedRun, c3_lengths  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=60)
    ap.add_argument("--threads", type=int, default=15)
    ap.add_argument("--mode", default="both")
    ap.add_argument("--window-gib", type=int, default=48)
    ap.add_argument("--sha-prio", type=int, default=None,
                    help="the windows' SHA-256 stream priority (-1 high, 1 low, 0 the library's; default: -1 with the lane)")
    a = ap.parse_args()
    D.set_device(0)
    L = c3_lengths(20000)
    idx = lpt_shard(L, 8)[0]
    ids, lens = [int(i) for i in idx], [L[i] for i in idx]
    order = np.argsort(-np.asarray(lens), kind="stable")
    for mode in (("alone", "windows") if a.mode == "both" else (a.mode,)):
        if mode == "alone":  # the K longest blobs only, all through the lane
            pick = sorted(order[:a.k].tolist())
            wr = WindowedRun(D, [ids[i] for i in pick], [lens[i] for i in pick], 4 << 20, a.window_gib << 30,
                             host_lane=(a.k, a.threads))
        else:
            wr = WindowedRun(D, ids, lens, 4 << 20, a.window_gib << 30, host_lane=(a.k, a.threads),
                             sha_priority=a.sha_prio)
        t0 = time.perf_counter()
        wr.run()
        el = time.perf_counter() - t0
        hb = sum(wr.lens[i] for i in wr.lane_blobs)
        print(f"{mode}: sha_prio={a.sha_prio} K={a.k} T={a.threads}: run {el:.2f} s, "
              f"lane {wr.lane_seconds:.2f} s = "
              f"{hb / wr.lane_seconds / 1e9:.2f} GB/s ({hb / wr.lane_seconds / 1e9 / a.threads:.2f} a thread), "
              f"{len(wr.wins)} windows", flush=True)
        wr.close()


if __name__ == "__main__":
    main()
