"""Concurrent GPU Digesters through the submission engine (engine.cpp), outside pytest:
N digesters on N threads, L bytes each, random write sizes; prints the aggregate and
per-stream rate and the streams per SHA launch.  KRK_ENGINE_TRACE=1 adds one stderr
line per SHA launch (size, why it was formed, launches in flight, the per-byte estimate).

    python tools/engine_probe.py [--n 256] [--mib 16] [--rounds 2]
"""
import argparse
import ctypes as C
import hashlib
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kraken_amd import core, device as D  # noqa: E402
from kraken_amd._capi import KRK_PLACE_GPU, check, lib  # noqa: E402


def stats():
    v = [C.c_uint64() for _ in range(5)]
    check(lib.krk_engine_stats(*[C.byref(x) for x in v]))
    return [x.value for x in v]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--mib", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--max-write", type=int, default=1 << 20)
    a = ap.parse_args()
    D.set_device(0)
    n, L = a.n, a.mib << 20
    base = np.random.default_rng(256).integers(0, 256, L + n * 4096, dtype=np.uint8).tobytes()
    datas = [memoryview(base)[i * 4096: i * 4096 + L] for i in range(n)]
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda m: hashlib.sha256(m).hexdigest(), datas))

    import threading
    bar = [threading.Barrier(n + 1)]

    def work(i):
        r = np.random.default_rng(i)
        d = core.Digester(KRK_PLACE_GPU)
        m, pos = datas[i], 0
        bar[0].wait()  # the uploads start together
        while pos < L:
            k = min(L - pos, int(r.integers(1, a.max_write)))
            d._write(m[pos:pos + k])
            pos += k
        return d.Digest().Hex()

    for rnd in range(a.rounds):
        bar[0] = threading.Barrier(n + 1)
        b0 = stats()
        with ThreadPoolExecutor(n) as ex:
            futs = [ex.submit(work, i) for i in range(n)]
            bar[0].wait()  # timed from the moment every thread holds its digester
            t0 = time.perf_counter()
            got = [f.result() for f in futs]
            el = time.perf_counter() - t0
        b1 = stats()
        assert got == want
        agg = n * L / el
        print(f"round {rnd}: {n} digesters x {a.mib} MiB: {el:.3f} s, {agg / 1e9:.2f} GB/s, "
              f"{agg / n / 1e6:.1f} MB/s a stream, {(b1[1] - b0[1]) / max(1, b1[0] - b0[0]):.1f} streams/launch, "
              f"{b1[0] - b0[0]} launches, pinned {b1[4] >> 20} MiB", flush=True)


if __name__ == "__main__":
    main()
