"""What a windowed host offload could buy C3, from the window plan
itself: the run is the sum over windows of (the window's largest chunk / the per-stream
rate of its launch plan), so handing the K longest blobs to host threads (SHA-NI, ~33 GB/s
on a 16-core share, their bytes read out of HBM) shortens it only as much as the next
longest blobs are shorter -- and C3's lengths are uniform up to 1.0736 GB.

Per-stream rates: 51.6 MB/s two lanes (> 4,096 live streams), 58 MB/s eight lanes, the
round-2 measurements; 0.5 ms a window of launch overhead.

    python tools/c3_offload_model.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kraken_amd.shard import lpt_shard  # noqa: E402
from kraken_amd.windowed import c3_lengths, window_plan  # noqa: E402

HOST_BPS = 33e9  # 16 host threads x ~2.1 GB/s SHA-NI (planner rates, profiles/r03)


def run_seconds(lens, W=48 << 30, cap=14336):
    t = 0.0
    wins = window_plan(lens, W, cap)
    for blobs, offs, take in wins:
        r = 58e6 if len(blobs) <= 4096 else 51.6e6
        t += float(take.max()) / r + 0.0005
    return t, len(wins)


def main():
    L = c3_lengths(20000)
    for tag, lens, ks in (("N=1 (20,000 blobs)", L, (0, 100, 200, 322, 500, 800)),
                          ("rank 0 of 8 (LPT shard)", [L[i] for i in lpt_shard(L, 8)[0]], (0, 20, 40, 80, 120, 200))):
        order = np.argsort(-np.asarray(lens))
        for k in ks:
            rest = [lens[i] for i in order[k:]]
            hb = sum(lens[i] for i in order[:k])
            t, n = run_seconds(rest)
            print(f"{tag}: K={k:4d} longest on the host ({hb / 1e9:7.1f} GB, {hb / HOST_BPS:5.1f} s of host time) "
                  f"-> GPU windows {t:6.2f} s ({n} windows)")


if __name__ == "__main__":
    main()
