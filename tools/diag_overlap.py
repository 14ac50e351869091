"""Do the SHA-256 and piece-CRC launches of one step overlap on the device?

Prints the hipEvent timeline (krk_kernel_timeline) of the SHA, CRC and synth launches
of a C3-shaped windowed run (scaled lengths, production live cap) and of a C2-shaped
krk_metainfo_digest_dev step, in this process.  --extra-streams N creates N more HIP
streams first (as a process with the submission engine running has).
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kraken_amd import device as D  # noqa: E402
from kraken_amd.windowed import WindowedRun, c3_lengths  # noqa: E402


def show(tag, k):
    tl = D.KernelTimer.timeline(k)
    for i, (plan, units, a, b) in enumerate(tl[:8]):
        print(f"{tag} {k:13s} #{i} plan={plan} units={units} start={a:9.3f} end={b:9.3f} dur={b - a:8.3f}")


def overlap_count():
    """Windows whose CRC launch ended before their SHA launch did (ran beside it)."""
    sha = D.KernelTimer.timeline("sha256_multi")
    crc = D.KernelTimer.timeline("crc32_pieces")
    inside = sum(1 for s, c in zip(sha, crc) if c[3] <= s[3])
    return inside, min(len(sha), len(crc))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extra-streams", type=int, default=0)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--window-gib", type=int, default=16)
    a = ap.parse_args()
    D.set_device(0)
    extra = []
    for _ in range(a.extra_streams):
        s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(s)))
        extra.append(s)
    lens = c3_lengths(a.n, scale=64)
    ids = [(2 << 40) + i for i in range(a.n)]
    wr = WindowedRun(D, ids, lens, 4 << 20, a.window_gib << 30)
    wr.run()  # warm
    wr.close()
    wr = WindowedRun(D, ids, lens, 4 << 20, a.window_gib << 30)
    with D.KernelTimer():
        wr.run()
        for k in ("sha256_multi", "crc32_pieces", "synth_fill"):
            show("c3", k)
        print("c3 CRC inside SHA: %d of %d windows (KRK_STREAM_MODE=%s)" % (*overlap_count(),
                                                                          os.environ.get("KRK_STREAM_MODE", "0")))
    wr.close()
    n = 1000
    arena = D.BlobArena([16 << 20] * n, 4 << 20, blob_ids=range(n))
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    with D.KernelTimer():
        D.metainfo_digest(arena, out)
        D.synchronize()
        for k in ("sha256_multi", "crc32_pieces"):
            show("c2", k)


if __name__ == "__main__":
    main()
