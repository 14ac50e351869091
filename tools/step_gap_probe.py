"""Host time inside one bench step (C2 shape): where the gap between one step's last
kernel and the next step's first command goes (development tool).

Prints, per step, the wall time of each phase: the metainfo_digest call (enqueue),
synchronize (wait for the kernels), the two D2H result copies.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kraken_amd import device as D  # noqa: E402


def main():
    n, mb = int(os.environ.get("N", 1000)), int(os.environ.get("MB", 100))
    pieces_only = os.environ.get("PIECES") == "1"  # C4 shape: N=1 MB=20480 PL=262144 PIECES=1
    D.set_device(0)
    lens = [mb << 20] * n
    arena = D.BlobArena(lens, int(os.environ.get("PL", 4 << 20)), blob_ids=list(range(n)))
    out = D.BatchOutputs(arena)
    pin_s = D.PinnedArray((arena.total_pieces,), np.uint32)
    pin_d = D.PinnedArray((n * 32,), np.uint8)
    timing = os.environ.get("TIMING", "1") == "1"
    for k in range(int(os.environ.get("STEPS", 4))):
        if timing:
            D.lib.krk_set_timing(1)
        t0 = time.perf_counter()
        if pieces_only:
            D.piece_sums(arena, out)
        else:
            D.metainfo_digest(arena, out)
        t1 = time.perf_counter()
        D.synchronize()
        t2 = time.perf_counter()
        pin_s.fill_from(out.sums)
        t3 = time.perf_counter()
        pin_d.fill_from(out.digests)
        t4 = time.perf_counter()
        if timing:
            D.KernelTimer.stats("crc32_pieces" if pieces_only else "sha256_multi")
        t5 = time.perf_counter()
        print(json.dumps({"step": k, "timing": timing, "enqueue_ms": round((t1 - t0) * 1e3, 3),
                          "sync_ms": round((t2 - t1) * 1e3, 3), "d2h_sums_ms": round((t3 - t2) * 1e3, 3),
                          "d2h_digests_ms": round((t4 - t3) * 1e3, 3), "stats_ms": round((t5 - t4) * 1e3, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
