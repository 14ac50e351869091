"""Tail-handoff thread rate probe: T Python threads each continue a
SHA-256 chain on the host from device bytes (krk_sha256_resume_dev_on_host, 64 MiB runs of
one 256 MiB device buffer a thread) for a few seconds -- alone, and beside a long SHA-256
launch of 2,500 eight-lane streams (the shape of an 8-GPU C3 shard's windows).  Prints one
JSON line per case: per-thread and total GB/s, and the process CPU seconds per wall second
(a CPU quota throttles above it)."""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kraken_amd import device as D  # noqa: E402
from kraken_amd.windowed import _IV  # noqa: E402

D.set_device(0)
BUF = 256 << 20
RUN = 64 << 20


def threads_rate(T, secs, bufs, idle):
    stop = time.perf_counter() + secs
    done = [0] * T

    def work(i):
        D.set_device(0)
        h = _IV.copy()
        off = 0
        while time.perf_counter() < stop:
            o = off % BUF
            D.check(D.lib.krk_sha256_resume_dev_on_host(h.ctypes.data_as(C.POINTER(C.c_uint32)), off,
                                                        C.c_void_p(bufs[i].ptr + o), RUN, 0, None, None))
            off += RUN
            done[i] += RUN

    c0 = time.process_time()
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    cpu = time.process_time() - c0
    return {"threads": T, "GBps_total": round(sum(done) / el / 1e9, 2),
            "GBps_per_thread": round(sum(done) / el / 1e9 / T, 3), "cpu_per_wall": round(cpu / el, 2)}


def main():
    Tmax = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    bufs = [D.DeviceBuffer(BUF) for _ in range(Tmax)]
    idle = []
    for b in bufs:
        D.check(D.lib.krk_synth_fill_dev(b.ptr, 7, 0, BUF, 0, None))
        s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(s)))
        idle.append(s)
    D.synchronize()
    for T in (1, 8, 12, Tmax):
        print(json.dumps({"case": "alone", **threads_rate(T, 3.0, bufs, idle)}), flush=True)
    # beside a long SHA-256 launch: 2,500 streams x 160 MiB of one shared buffer (eight lanes,
    # ~2.7 s at ~59 MB/s a stream), on a high-priority stream like the windows'
    n, L = 2500, 160 << 20
    big = D.DeviceBuffer(L)
    D.check(D.lib.krk_synth_fill_dev(big.ptr, 9, 0, L, 0, None))
    ptrs = (C.c_void_p * n)(*([big.ptr] * n))
    lens = np.full(n, L, dtype=np.uint64)
    dig = D.DeviceBuffer(32 * n)
    hs = C.c_void_p()
    D.check(D.lib.krk_stream_create_prio(-1, C.byref(hs)))
    for T in (8, Tmax):
        D.check(D.lib.krk_sha256_dev(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), n, C.c_void_p(dig.ptr), hs))
        time.sleep(0.05)
        r = threads_rate(T, 2.0, bufs, idle)
        t0 = time.perf_counter()
        D.check(D.lib.krk_stream_sync(hs))
        print(json.dumps({"case": "beside_sha_launch", **r, "sha_left_s": round(time.perf_counter() - t0, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
