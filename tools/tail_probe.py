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
    print(json.dumps({"case": "alone", **threads_rate(Tmax, 2.0, bufs, idle)}), flush=True)
    # beside a long SHA-256 launch: 2,500 streams x 160 MiB of one shared buffer (eight lanes,
    # ~2.7 s at ~59 MB/s a stream), on a high-priority stream like the windows'
    n, L = 2500, 320 << 20
    big = D.DeviceBuffer(L)
    D.check(D.lib.krk_synth_fill_dev(big.ptr, 9, 0, L, 0, None))
    ptrs = (C.c_void_p * n)(*([big.ptr] * n))
    lens = np.full(n, L, dtype=np.uint64)
    dig = D.DeviceBuffer(32 * n)
    hs = C.c_void_p()
    D.check(D.lib.krk_stream_create_prio(-1, C.byref(hs)))
    # what else runs beside the C3 windows: a 10 GiB generator launch every 70 ms on a normal
    # stream (waited for by the host), CRC launches of 2.5 GB on a high-priority stream, a
    # thread polling events every 2 ms
    gbuf = D.DeviceBuffer(10 << 30)
    gs, cs = C.c_void_p(), C.c_void_p()
    D.check(D.lib.krk_stream_create(C.byref(gs)))
    D.check(D.lib.krk_stream_create_prio(-1, C.byref(cs)))
    cb = D.ChunkedBatch([40 * (64 << 20)], 4 << 20)

    def gen_loop(stop):
        while not stop.is_set():
            D.check(D.lib.krk_synth_fill_dev(gbuf.ptr, 11, 0, 10 << 30, 0, gs))
            D.check(D.lib.krk_stream_sync(gs))
            time.sleep(0.065)

    def crc_loop(stop):
        ptr = np.array([gbuf.ptr + k * (64 << 20) for k in range(40)], dtype=np.uint64)
        off = np.arange(40, dtype=np.uint64) * np.uint64(64 << 20)
        ln = np.full(40, 64 << 20, dtype=np.uint64)
        while not stop.is_set():
            arr = D.chunk_array(ptr, off, ln, cb.lengths[0], cb.piece_lengths[0], cb.sums_off[0], np.uint64(0))
            D.check(D.lib.krk_chunks_crc_dev(arr.ctypes.data_as(C.POINTER(D.krk_chunk)), 40, cb.sums.ptr, cs))
            D.check(D.lib.krk_stream_sync(cs))
            time.sleep(0.07)

    def poll_loop(stop):
        e = C.c_void_p()
        D.check(D.lib.krk_event_create(C.byref(e)))
        D.check(D.lib.krk_event_record(e, hs))
        done = C.c_int()
        while not stop.is_set():
            D.check(D.lib.krk_event_query(e, C.byref(done)))
            time.sleep(0.002)

    for case, loops in (("beside_sha_launch", []), ("+gen", [gen_loop]), ("+crc", [crc_loop]),
                        ("+poll", [poll_loop]), ("+all", [gen_loop, crc_loop, poll_loop])):
        D.check(D.lib.krk_sha256_dev(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), n, C.c_void_p(dig.ptr), hs))
        stop = threading.Event()
        th = [threading.Thread(target=f, args=(stop,)) for f in loops]
        for t in th:
            t.start()
        time.sleep(0.05)
        r = threads_rate(Tmax, 2.0, bufs, idle)
        stop.set()
        for t in th:
            t.join()
        t0 = time.perf_counter()
        D.check(D.lib.krk_stream_sync(hs))
        print(json.dumps({"case": case, **r, "sha_left_s": round(time.perf_counter() - t0, 3)}), flush=True)


if __name__ == "__main__":
    main()
