"""End-to-end (host buffers -> PCIe -> both kernels) probe: the bench's e2e leg
(1,000 blobs x 16 MiB of the C2 synthetic content in pageable host memory) at
several staging window sizes, with the library's host phase trace (KRK_TRACE=1).
Development tool, not the bench contract."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blobs", type=int, default=1000)
    ap.add_argument("--mb", type=int, default=16)
    ap.add_argument("--windows", default="256,512,1024")
    ap.add_argument("--sha-only", action="store_true")
    a = ap.parse_args()
    os.environ["KRK_TRACE"] = "1"
    from kraken_amd import device as D
    D.set_device(0)
    L, P = a.mb << 20, 4 << 20
    datas = [np.empty(L, dtype=np.uint8) for _ in range(a.blobs)]
    import ctypes as C
    arena = D.BlobArena([L] * a.blobs, P)
    for i, d in enumerate(datas):
        D.check(D.lib.krk_memcpy_d2h(d.ctypes.data_as(C.c_void_p), arena.buf.ptr + int(arena.offsets[i]), L))
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    ref = out.digests.to_host(np.uint8, 32 * a.blobs).reshape(-1, 32)
    del arena
    for wmb in [int(x) for x in a.windows.split(",")]:
        os.environ["KRK_WINDOW_MB"] = str(wmb)
        D.metainfo_digest_host(datas[:2], P)
        t0 = time.perf_counter()
        sums, dg = D.metainfo_digest_host(datas, P)
        el = time.perf_counter() - t0
        ok = bool(np.array_equal(dg, ref))
        print(json.dumps({"window_mb": wmb, "seconds": round(el, 3), "GBps": round(a.blobs * L / el / 1e9, 2),
                          "digests_match_device": ok}), flush=True)


if __name__ == "__main__":
    main()
