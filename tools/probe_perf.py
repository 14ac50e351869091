"""Quick kernel throughput probe (development tool, not the bench contract).

Times the CRC piece kernel on a large device-resident arena and the SHA-256
kernel at several stream counts, with hipEvents recorded on the kernel stream.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kraken_amd import device as D  # noqa: E402


def crc(nbytes_gb: float, blob_mb: int, piece: int, reps: int):
    n = int(nbytes_gb * 1e9 / (blob_mb << 20))
    arena = D.BlobArena([blob_mb << 20] * n, piece)
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)
    D.synchronize()
    with D.KernelTimer():
        t0 = time.perf_counter()
        for _ in range(reps):
            D.piece_sums(arena, out)
        D.synchronize()
        t1 = time.perf_counter()
        k, ms = D.KernelTimer.stats("crc32_pieces")
    total = n * (blob_mb << 20)
    return {"what": "crc", "blobs": n, "bytes": total, "piece": piece, "wall_GBps": total * reps / (t1 - t0) / 1e9,
            "kernel_ms": ms / max(k, 1), "kernel_GBps": total / (ms / max(k, 1) / 1e3) / 1e9}


def crc_concurrent(n: int, mb: int, piece: int):
    """C2-sized arena: CRC alone, SHA alone, then both via metainfo_digest."""
    arena = D.BlobArena([mb << 20] * n, piece)
    out = D.BatchOutputs(arena)
    res = {"what": "c2_split", "blobs": n, "mb": mb}
    for name, fn in (("crc_alone", D.piece_sums), ("sha_alone", D.sha256), ("both", D.metainfo_digest)):
        with D.KernelTimer():
            t0 = time.perf_counter()
            fn(arena, out)
            D.synchronize()
            t1 = time.perf_counter()
            k1, ms1 = D.KernelTimer.stats("crc32_pieces")
            k2, ms2 = D.KernelTimer.stats("sha256_multi")
        res[name] = {"wall_ms": round((t1 - t0) * 1e3, 2), "crc_ms": round(ms1, 3), "sha_ms": round(ms2, 2)}
    return res


def sha(streams: int, mb: int):
    arena = D.BlobArena([mb << 20] * streams, 1 << 20)
    out = D.BatchOutputs(arena)
    with D.KernelTimer():
        t0 = time.perf_counter()
        D.sha256(arena, out)
        D.synchronize()
        t1 = time.perf_counter()
        k, ms = D.KernelTimer.stats("sha256_multi")
    total = streams * (mb << 20)
    return {"what": "sha", "streams": streams, "mb": mb, "kernel_ms": ms, "GBps": total / (ms / 1e3) / 1e9,
            "per_stream_MBps": (mb << 20) / (ms / 1e3) / 1e6, "wall_s": t1 - t0}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--crc-gb", type=float, default=16)
    ap.add_argument("--sha", default="64:8,1024:8,4096:4,16384:1")
    ap.add_argument("--variant", default="16", help="KRK_CRC_VARIANT (production: 7, 8, 14-17; default 16)")
    ap.add_argument("--sha-plan", type=int, default=0,
                    help="krk_set_sha_plan: 0 auto, 1-4 production, 100-107 diagnostics (KRK_DIAG build, "
                         "KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so)")
    ap.add_argument("--c2", action="store_true")
    ap.add_argument("--split", default="", help="n:blob_mb:piece_kb,... CRC alone / SHA alone / both (c2_split shape)")
    ap.add_argument("--crc-spec", default="", help="gb:blob_mb:piece_kb,... custom CRC shapes")
    a = ap.parse_args()
    os.environ["KRK_CRC_VARIANT"] = a.variant
    D.set_device(0)
    D.check(D.lib.krk_set_sha_plan(a.sha_plan))
    res = []
    if a.c2:
        print(json.dumps(crc_concurrent(1000, 100, 4 << 20)), flush=True)
        sys.exit(0)
    if a.split:
        for spec in a.split.split(","):
            n, mb, pk = map(int, spec.split(":"))
            print(json.dumps(dict(crc_concurrent(n, mb, pk << 10), plan=a.sha_plan)), flush=True)
        sys.exit(0)
    if a.crc_spec:
        for spec in a.crc_spec.split(","):
            gb, mb, pk = spec.split(":")
            print(json.dumps(crc(float(gb), int(mb), int(pk) << 10, 3)), flush=True)
        sys.exit(0)
    if a.crc_gb > 0:
        res.append(crc(a.crc_gb, 100, 4 << 20, 3))
        print(json.dumps(res[-1]), flush=True)
        res.append(crc(4, 256, 256 << 10, 3))
        print(json.dumps(res[-1]), flush=True)
    if a.sha == "none":
        sys.exit(0)
    for spec in a.sha.split(","):
        s, mb = map(int, spec.split(":"))
        res.append(sha(s, mb))
        print(json.dumps(res[-1]), flush=True)
