"""Fluid model of C3 at N=1 on a mixed SHA-256 plan ("why C3 at N=1 stays at
~552 GB/s"): the K longest blobs run on eight lanes a stream from window 0, the rest on two
lanes, admitted longest first into the CUs the eight-lane workgroups leave.

Per-stream rates are the measured ones (eight lanes 58 MB/s, two lanes 52 MB/s in C3's
windows); a CU carries `c8` eight-lane or `c2` two-lane streams (LDS-limited: 16 / 64 with
today's 65 / 64 KiB pairs), 224 of the 256 CUs hold SHA-256 workgroups (an eighth stays free
for the window's CRC launch).  Time advances in `dt` steps; the job ends when every blob's
chain has.  Unlike the SIMD-time bound of the earlier estimate this model keeps the schedule's
tail: once the waiting blobs are admitted the windows empty and the longest chains run alone.

    python tools/sim_mixed_plan.py            # K sweep, today's LDS footprints
    python tools/sim_mixed_plan.py --c8 24    # eight-lane pairs small enough for 3 a CU
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from kraken_amd.windowed import c3_lengths  # noqa: E402


def simulate(L, K, c8=16, c2=64, r8=58e6, r2=52e6, cus=224, dt=0.02):
    """Seconds until every chain ends with the K longest blobs (L sorted descending) on eight lanes."""
    left = L.astype(np.float64).copy()
    fast = np.zeros(L.size, bool)
    fast[:K] = True
    live = fast.copy()
    nxt, t = K, 0.0
    rate = np.where(fast, r8, r2)
    while True:
        live &= left > 0
        k8 = int((live & fast).sum())
        cap2 = int(c2 * (cus - k8 / c8))
        n2 = int((live & ~fast).sum())
        if n2 < cap2 and nxt < L.size:
            add = min(cap2 - n2, L.size - nxt)
            live[nxt:nxt + add] = True
            nxt += add
        if not live.any() and nxt >= L.size:
            return t
        left[live] -= rate[live] * dt
        t += dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c8", type=int, default=16, help="eight-lane streams a CU")
    ap.add_argument("--c2", type=int, default=64, help="two-lane streams a CU")
    ap.add_argument("--ks", default="0,256,512,768,1024,1536,2048")
    a = ap.parse_args()
    L = np.sort(np.asarray(c3_lengths(20000), dtype=np.float64))[::-1]
    base = None
    for K in [int(x) for x in a.ks.split(",")]:
        t = simulate(L, K, a.c8, a.c2)
        base = base or t
        print(f"K={K:5d}  {t:6.2f} s  {L.sum() / t / 1e9:6.1f} GB/s  gain {base / t:.3f}")


if __name__ == "__main__":
    main()
