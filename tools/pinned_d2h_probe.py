"""Device-to-host copy rate into page-locked buffers by allocator:
64 MiB copies on one stream from HBM into (a) krk_host_alloc buffers (mmap + transparent huge
pages + hipHostRegister, pages placed by the allocating thread's first touch) and (b)
hipHostMalloc (krk_host_alloc_dma's allocator), with the NUMA node of each buffer's first page
(move_pages).  Prints one JSON line per case."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kraken_amd import device as D  # noqa: E402

PIECE = 64 << 20
NBUF = int(sys.argv[1]) if len(sys.argv) > 1 else 8
libc = C.CDLL(None, use_errno=True)


def numa_node(addr):
    pages = (C.c_void_p * 1)(addr)
    status = (C.c_int * 1)(-99)
    r = libc.syscall(279, 0, 1, pages, None, status, 0)  # move_pages(pid 0, query only)
    return int(status[0]) if r == 0 else None


def rate(ptrs, src, s, reps=6):
    for p in ptrs:  # warm
        D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(p), C.c_void_p(src.ptr), PIECE, s))
    D.check(D.lib.krk_stream_sync(s))
    t0 = time.perf_counter()
    for _ in range(reps):
        for p in ptrs:
            D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(p), C.c_void_p(src.ptr), PIECE, s))
    D.check(D.lib.krk_stream_sync(s))
    return reps * len(ptrs) * PIECE / (time.perf_counter() - t0) / 1e9


def main():
    D.set_device(0)
    src = D.DeviceBuffer(PIECE)
    D.check(D.lib.krk_synth_fill_dev(src.ptr, 3, 0, PIECE, 0, None))
    s = C.c_void_p()
    D.check(D.lib.krk_stream_create(C.byref(s)))
    D.synchronize()
    cases = {}
    lib_bufs = [D.PinnedArray((PIECE,), np.uint8) for _ in range(NBUF)]
    cases["krk_host_alloc"] = [b.ptr for b in lib_bufs]
    hip = C.CDLL(D.lib._name)  # the HIP runtime the library itself loaded
    hm = []
    for _ in range(NBUF):
        p = C.c_void_p()
        assert hip.hipHostMalloc(C.byref(p), C.c_size_t(PIECE), 0) == 0
        C.memset(p, 1, PIECE)
        hm.append(p.value)
    cases["hipHostMalloc"] = hm
    for name, ptrs in cases.items():
        nodes = [numa_node(p) for p in ptrs]
        per = [round(rate([p], src, s, reps=2), 1) for p in ptrs]  # each buffer alone
        print(json.dumps({"case": name, "buffers": len(ptrs), "GBps": round(rate(ptrs, src, s, reps=2), 2),
                          "numa_nodes": {str(n): nodes.count(n) for n in sorted(set(nodes), key=str)},
                          "per_buffer_GBps_min_median_max": [min(per), sorted(per)[len(per) // 2], max(per)],
                          "slow_buffers_below_40": sum(x < 40 for x in per),
                          "slow_by_node": {str(n): sum(1 for x, m in zip(per, nodes) if x < 40 and m == n)
                                           for n in sorted(set(nodes), key=str)}}), flush=True)


if __name__ == "__main__":
    main()
