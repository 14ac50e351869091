"""Larger-than-HBM batches (config C3: 20k blobs of 100 MiB-1 GiB, ~1.47 TB per GPU
against 288 GB of HBM): every live blob advances by one chunk per device window
through krk_metainfo_digest_chunks_dev -- SHA-256 from per-blob midstates in HBM,
piece CRCs XOR-accumulated by byte range -- while the next window is generated
(synthetic data) on its own stream.

This is the machinery bench.py's C3 line runs and tests/test_gpu_windowed.py checks
against the oracle and the one-shot path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def c3_lengths(n_total=20000, scale: int = 1):
    """L_i = 104,857,600 + (rng_i mod 968,884,225), rng_i = mix64(0xC3 + i*gamma)
    (SURVEY.md 8(d) C3); `scale` > 1 divides every length (same law, smaller bytes)."""
    return [(104_857_600 + mix64((0xC3 + i * GAMMA) & M64) % 968_884_225) // scale for i in range(n_total)]


def window_plan(lens, W, cap):
    """Windows: [(blob indices, offsets, chunk lengths)] -- the library's window schedule
    (krk_window_sched_*, kraken_amd/csrc/windows.cpp; the same one its host-resident batch
    calls run).  Every live blob advances by the same 64-multiple chunk per window (about W
    bytes a window).  Admission: at most `cap` blobs are live, admitted longest first, so the
    longest chain starts in window 0 and every window stays on a multi-lane SHA plan (eight
    lanes a stream up to 16 x CUs live streams, two up to 64 x CUs; a launch of more streams
    falls back to one lane per stream, ~0.7x per stream); a finished blob's
    slot goes to the next-longest waiting blob."""
    from ._capi import check, lib
    L = np.ascontiguousarray(lens, dtype=np.uint64)
    n = L.size
    if n == 0:
        return []
    cap = max(1, min(int(cap), n))
    h = C.c_void_p()
    check(lib.krk_window_sched_new(L.ctypes.data_as(C.POINTER(C.c_uint64)), n, int(W), cap, C.byref(h)))
    wins = []
    try:
        b = np.zeros(cap, dtype=np.uint32)
        o = np.zeros(cap, dtype=np.uint64)
        t = np.zeros(cap, dtype=np.uint64)
        k = C.c_uint64(0)
        while True:
            check(lib.krk_window_sched_next(h, b.ctypes.data_as(C.POINTER(C.c_uint32)),
                                            o.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            t.ctypes.data_as(C.POINTER(C.c_uint64)), cap, C.byref(k)))
            if not k.value:
                break
            m = k.value
            wins.append((b[:m].astype(np.int64), o[:m].copy(), t[:m].copy()))
    finally:
        lib.krk_window_sched_free(h)
    return wins


def two_lane_stream_cap(D, n):
    """Largest stream count <= n whose SHA launch plan runs a stream on more than one
    lane (eight or two lanes per stream; the one-lane plan's chain is the slowest)."""
    if n == 0 or D.sha_lanes_per_stream(n) >= 2:
        return max(n, 1)
    lo, hi = 1, n  # several lanes at lo, one at hi
    if D.sha_lanes_per_stream(lo) < 2:
        return n
    while hi - lo > 1:
        mid = (lo + hi) // 2
        lo, hi = (mid, hi) if D.sha_lanes_per_stream(mid) >= 2 else (lo, mid)
    return lo


def window_stream_cap(D, n):
    """Live streams per window: at most 7/8 of the largest multi-lane stream count (a
    multiple of the two-pair workgroup's 64; krk_window_stream_cap, the cap the library's
    host-resident windows use too).  At the full two-lane count (64 x CUs) every CU holds a
    128 KiB SHA workgroup and the window's piece-CRC launch (144 KiB workgroups) waits for
    the SHA launch to end; with an eighth of the CUs left free it runs inside it, and the
    chain of the longest blob -- not the live count -- still sets the run time.  C3 on one
    MI355X (bench --live-cap): 16,384 live 494 GB/s, 15,360 522, 14,336 524, 13,824 523,
    13,312 522, 12,288 509 (profiles/r02/c3_live_cap.jsonl)."""
    v = C.c_uint64(0)
    D.check(D.lib.krk_window_stream_cap(C.byref(v)))
    return max(1, min(n, v.value))


def stream_rate(rates, n_streams):
    """One SHA-256 stream's rate (B/s) in a launch of n_streams: the planner rate of the
    AUTO tier the launch falls in (eight lanes up to 16 x CUs streams, two lanes up to
    64 x CUs, one lane beyond; krk_planner_rates)."""
    cus = max(1, int(rates["cus"]))
    return rates["sha_stream_bps"][0 if n_streams <= 16 * cus else 1 if n_streams <= 64 * cus else 2]


def windows_seconds(rates, lens, W, cap, launch_s=0.0005):
    """Modelled run time of the windows over `lens`: each window lasts its largest chunk
    at the per-stream rate of its launch plan (the chain of the window's longest chunk
    sets it), plus a launch overhead."""
    t = 0.0
    for blobs, _, take in window_plan(lens, W, cap):
        t += float(take.max()) / stream_rate(rates, blobs.size) + launch_s
    return t


def host_lane_plan(D, lens, W, cap, threads, rates=None, min_gain=0.02):
    """How many of the longest blobs the host lane takes: K (a multiple of `threads`, the
    lane hashes one group of `threads` blobs at a time) minimising max(GPU windows over the
    rest, host groups), from the planner rates (krk_planner_rates: per-stream rates
    measured on the device, one host thread's SHA-256 rate, the D2H rate shared by the
    threads).  0 unless it shortens the modelled run by min_gain.  Returns (K, modelled
    seconds with it, modelled seconds without)."""
    rates = rates or D.planner_rates()
    T = max(1, int(threads))
    L = np.asarray(lens, dtype=np.int64)
    order = np.argsort(-L, kind="stable")
    per_thread = min(rates["host_sha_bps"], rates["d2h_bps"] / T)

    def cost(m):  # m groups of T on the host
        k = min(m * T, L.size)
        host = sum(float(L[order[g * T]]) / per_thread for g in range(m))  # a group lasts its longest blob
        rest = L[order[k:]]
        gpu = windows_seconds(rates, rest, W, min(cap, max(1, rest.size))) if rest.size else 0.0
        return max(gpu, host), k

    base, _ = cost(0)
    lo, hi = 0, (L.size + T - 1) // T
    while hi - lo > 2:  # max(decreasing, increasing): ternary search on the group count
        m1, m2 = lo + (hi - lo) // 3, hi - (hi - lo) // 3
        if cost(m1)[0] <= cost(m2)[0]:
            hi = m2
        else:
            lo = m1
    best, k = min(cost(m) for m in range(lo, hi + 1))
    if best > base * (1 - min_gain):
        return 0, base, base
    return k, best, base


def lane_groups(lens, k, threads):
    """The host lane's blobs: the K longest (sorted indices) and the groups of `threads`
    of them it hashes one after the other, longest first.  The last group stops at K (it
    once ran on into the window blobs, hashing them too and zeroing the piece sums the
    windows had accumulated for them)."""
    L = np.asarray(lens, dtype=np.int64)
    k = int(min(max(k, 0), L.size))
    T = max(1, int(threads))
    order = np.argsort(-L, kind="stable")
    blobs = np.sort(order[:k]) if k else np.zeros(0, dtype=np.int64)
    return blobs, [order[g:min(g + T, k)] for g in range(0, k, T)]


class WindowedRun:
    """One batch of synthetic blobs (ids, lens, piece length P) streamed through two
    device windows of W bytes: window k+1 is generated on `gen` while window k's
    kernels run on `run`.  After run(): cb.sums / cb.digests hold every blob's piece
    sums and digest (device).

    host_lane=(K, threads): the K longest blobs skip the windows; a host-lane thread
    generates them `threads` at a time into a device buffer of their own, queues their
    piece CRCs on the GPU (krk_piece_sums_dev, into cb.sums) and hashes them on `threads`
    host threads (krk_sha256_dev_on_host: each reads a blob out of HBM through pinned
    double buffers), while the windows run the rest; their digests go into cb.digests at
    the end of run()."""

    def __init__(self, D, ids, lens, P, W, cap=None, host_lane=None, device=0, sha_priority=None):
        self.D = D
        self.ids = np.asarray(ids, dtype=np.uint64)
        self.lens = list(lens)
        self.P = P
        self.W = int(W)
        self.device = device
        n = len(self.lens)
        L = np.asarray(self.lens, dtype=np.int64)
        k, self.lane_threads = (host_lane or (0, 0))
        order = np.argsort(-L, kind="stable")
        self.lane_blobs, self.lane_groups = lane_groups(L, k, self.lane_threads)
        gpu = np.setdiff1d(np.arange(n), self.lane_blobs) if k else np.arange(n)
        self.cap = window_stream_cap(D, gpu.size) if cap is None else int(cap)
        self.wins = [(gpu[b], o, t) for b, o, t in window_plan(L[gpu], self.W, self.cap)]
        wb = self.W + 16 * max(gpu.size, 1)
        self.bufs = [D.DeviceBuffer(wb), D.DeviceBuffer(wb)] if self.wins else []
        self.lane_bufs, self.lane_ss = [], []
        if k:  # two buffers of a group each (the first group holds the longest blobs)
            nb = (int(L[order[0]]) + 256) * len(self.lane_groups[0])
            self.lane_bufs = [D.DeviceBuffer(nb) for _ in range(min(2, len(self.lane_groups)))]
        self.lane_digests = None
        self.lane_seconds = 0.0
        self.cb = D.ChunkedBatch(self.lens, P)
        self.gen_s, self.run_s, self.sha_s = C.c_void_p(), C.c_void_p(), C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(self.run_s)))
        D.check(D.lib.krk_stream_create(C.byref(self.gen_s)))
        # With the host lane, the windows' SHA-256 launches (up to ~0.6 s each) go on a
        # high-priority stream, i.e. hardware queues of their own: normal-priority streams
        # share GPU_MAX_HW_QUEUES queues, and the lane's D2H copies and generator / CRC
        # launches queued on a stream sharing the SHA launch's queue wait behind it.  Rank
        # 0's shard of an 8-GPU C3 (tools/lane_probe.py, 480 blobs on 15 threads): lane 24.3
        # s on the shared queues, 15.75 s with the SHA launches apart.  Without the lane they
        # stay on the library's stream (a C3 N=1 run measured 553 GB/s there, 499 with its
        # SHA launches at high priority).
        if sha_priority is None:
            sha_priority = -1 if k else 0
        if sha_priority and not self.sha_s.value:
            D.check(D.lib.krk_stream_create_prio(int(sha_priority), C.byref(self.sha_s)))
        for _ in self.lane_bufs:
            self.lane_ss.append(C.c_void_p())
            D.check(D.lib.krk_stream_create(C.byref(self.lane_ss[-1])))

    def _items(self, k):
        blobs, offs, take = self.wins[k]
        dev = np.zeros(take.size, dtype=np.uint64)  # 16-byte aligned chunk addresses in the window
        dev[1:] = np.cumsum((take + np.uint64(15)) // np.uint64(16) * np.uint64(16))[:-1]
        dev += np.uint64(self.bufs[k & 1].ptr)
        return blobs, dev, offs, take

    def _gen(self, items):
        blobs, dev, offs, take = items
        self.D.synth_fill_chunk_arrays(self.ids[blobs], dev, offs, take, stream=self.gen_s)
        self.D.check(self.D.lib.krk_stream_sync(self.gen_s))

    def _lane(self, err):
        """The host lane's thread: group by group (longest first), generate the group's
        blobs into one of two lane buffers and queue their piece CRCs on that buffer's
        stream, then hash the previous group on the host threads -- group g+1 is
        generated and CRC'd on the device while group g is hashed."""
        D = self.D
        try:
            import time
            t0 = time.perf_counter()
            D.set_device(self.device)
            dig = np.zeros((len(self.lens), 32), dtype=np.uint8)
            L = np.asarray(self.lens, dtype=np.uint64)

            def place(g, b):
                ln = L[g]
                dev = np.zeros(g.size, dtype=np.uint64)  # 256-byte aligned slots in lane buffer b
                dev[1:] = np.cumsum((ln + np.uint64(255)) // np.uint64(256) * np.uint64(256))[:-1]
                dev += np.uint64(self.lane_bufs[b].ptr)
                s = self.lane_ss[b]
                D.synth_fill_chunk_arrays(self.ids[g], dev, np.zeros(g.size, np.uint64), ln, stream=s)
                for j in range(g.size):  # one call a blob: a call zeroes the whole sums span it covers
                    D.piece_sums_dev_arrays(dev[j:j + 1], ln[j:j + 1], self.cb.piece_lengths[g[j:j + 1]],
                                            self.cb.sums_off[g[j:j + 1]], self.cb.sums.ptr, stream=s)
                return dev, ln

            groups = self.lane_groups
            cur = place(groups[0], 0)
            for k, g in enumerate(groups):
                # buffer (k+1)&1 last held group k-1: hashed (the call below is synchronous)
                # and CRC'd (same stream, earlier) before the next fill is queued behind them
                nxt = place(groups[k + 1], (k + 1) & 1) if k + 1 < len(groups) else None
                dig[g] = D.sha256_dev_on_host(cur[0], cur[1], self.lane_threads, stream=self.lane_ss[k & 1])
                cur = nxt
            for s in self.lane_ss:  # the last groups' CRCs
                D.check(D.lib.krk_stream_sync(s))
            self.lane_digests = dig
            self.lane_seconds = time.perf_counter() - t0
        except BaseException as e:  # re-raised on the caller's thread
            err.append(e)

    def run(self):
        """Window k's kernels are queued before the host waits for window k-1's (an
        event after each window), so the device goes from one window to the next with
        no host round trip; window k+1 is generated into k-1's buffer once k-1 is done.
        The host lane (if any) runs on its own thread meanwhile."""
        lane, err = None, []
        if self.lane_groups:
            import threading
            lane = threading.Thread(target=self._lane, args=(err,), name="krk-host-lane")
            lane.start()
        try:
            if self.wins:
                self._run_windows()
        finally:
            if lane is not None:
                lane.join()
        if err:
            raise err[0]
        if lane is not None:  # the lane's digests into the batch's digest rows
            D = self.D
            for i in self.lane_blobs:
                row = np.ascontiguousarray(self.lane_digests[i])
                D.check(D.lib.krk_memcpy_h2d(C.c_void_p(self.cb.digests.ptr + 32 * int(i)),
                                             row.ctypes.data_as(C.c_void_p), 32))

    def _run_windows(self):
        D = self.D
        cur = self._items(0)
        self._gen(cur)
        evs = [C.c_void_p(), C.c_void_p()]
        for e in evs:
            D.check(D.lib.krk_event_create(C.byref(e)))
        try:
            for k in range(len(self.wins)):
                self.cb.step_arrays(cur[0], cur[1], cur[2], cur[3], stream=self.run_s,
                                    sha_stream=self.sha_s if self.sha_s.value else None)
                D.check(D.lib.krk_event_record(evs[k & 1], self.run_s))
                if k + 1 < len(self.wins):
                    if k:  # window k-1 read buffer (k+1) & 1
                        D.check(D.lib.krk_event_sync(evs[(k - 1) & 1]))
                    cur = self._items(k + 1)
                    self._gen(cur)
            D.check(D.lib.krk_stream_sync(self.run_s))
        finally:
            for e in evs:
                D.lib.krk_event_destroy(e)

    def close(self):
        for b in self.bufs + self.lane_bufs:
            b.free()
        self.bufs, self.lane_bufs = [], []
        for s in [self.gen_s, self.run_s, self.sha_s] + self.lane_ss:
            if s.value:
                self.D.lib.krk_stream_destroy(s)
        self.gen_s, self.run_s, self.sha_s, self.lane_ss = C.c_void_p(), C.c_void_p(), C.c_void_p(), []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
