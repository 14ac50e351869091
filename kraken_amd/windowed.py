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


# ---------------------------------------------------------------------------------------
# Tail handoff of the windowed chains.  A windowed batch whose longest
# chain outlasts the GPU's aggregate work -- every shard of an 8-GPU C3, whose 1.07 GB blob
# takes ~18 s at ~58 MB/s a stream while the shard's 1.47 TB would take ~2 s -- ends when
# that chain ends.  Host threads (SHA-NI, ~2.3 GB/s, 40x a GPU stream) steal chains instead:
# at each window boundary every thread that will be free before the next window ends takes
# the chain with the most bytes left (earliest deadline first, as offload.cpp tail_plan does
# for batches in HBM), from the midstate the windows keep in HBM (ChunkedBatch.state); the
# chain leaves the window schedule (krk_window_sched_drop), its remaining bytes are
# generated on the device in 64 MiB pieces, their piece CRCs run on the GPU
# (krk_chunks_crc_dev, XOR-accumulated into the same sums), and the thread hashes them out
# of HBM (krk_sha256_resume_dev_on_host).  The threads start on the longest chains whole.
# The same policy is simulated on the planner's rates (simulate_tail_handoff): the bench
# reports that model beside the measured run.

_IV = np.array([0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19],
               dtype=np.uint32)
TAIL_PIECE = 64 << 20  # device bytes a tail thread generates, CRCs and hashes at a time
# Window chunk cap of the tail handoff: ~70 ms of a chain at eight lanes a window, so a
# chain is handed over within a short window of a thread becoming free, however few chains
# are left live (modelled on rank 0's shard of an 8-GPU C3: 1/2/4/8 MiB end at 11.7 / 11.7
# / 12.0 / 12.7 s with 0.5 ms a launch, 12.7 / 12.2 / 12.3 / 12.9 s with 3 ms).
TAIL_CHUNK = 4 << 20
# A thread gets its next chain while it is expected to be free within this many windows
# after the queued one ends: a chain handed over early idles on the GPU side (r/h ~ 2.4 % of
# the idle time in extra host bytes), a thread that finishes before the window holding its
# next chain's midstate ends waits for it (all of that time lost).
TAIL_HORIZON = 2.5
TAIL_RING = 8  # device slots a tail thread's pieces cycle through (generated / hashed / waiting for their CRC)
TAIL_FIRST_PIECE = 8 << 20  # a stolen chain's first piece (a multiple of 64)


def tail_thread_rate(rates, threads):
    """One tail thread's bytes/s: its SHA-NI rate (the planner's figure is derated 15 % for a
    loaded socket; a tail thread alone on its buffers loses ~2 %, offload.cpp tail_plan),
    capped by its share of the device-to-host copy rate."""
    return min(rates["host_sha_bps"] * (0.98 / 0.85), rates["d2h_bps"] / max(1, int(threads)))


class _Sched:
    """krk_window_sched over a subset of the batch (indices into the full batch)."""

    def __init__(self, lens, idx, W, cap, max_chunk=0):
        from ._capi import check, lib
        self.check, self.lib = check, lib
        self.idx = np.asarray(idx, dtype=np.int64)
        self.pos = {}
        L = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64)[self.idx])
        self.cap = max(1, min(int(cap), max(1, L.size)))
        self.h = C.c_void_p()
        if L.size:
            check(lib.krk_window_sched_new(L.ctypes.data_as(C.POINTER(C.c_uint64)), L.size, int(W), self.cap,
                                           C.byref(self.h)))
            if max_chunk:
                check(lib.krk_window_sched_set_chunk_cap(self.h, int(max_chunk)))
        self.sub = {int(b): k for k, b in enumerate(self.idx)}
        self._b = np.zeros(self.cap, dtype=np.uint32)
        self._o = np.zeros(self.cap, dtype=np.uint64)
        self._t = np.zeros(self.cap, dtype=np.uint64)

    def next(self):
        if not self.h.value:
            return None
        k = C.c_uint64(0)
        self.check(self.lib.krk_window_sched_next(self.h, self._b.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                  self._o.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                  self._t.ctypes.data_as(C.POINTER(C.c_uint64)), self.cap,
                                                  C.byref(k)))
        m = k.value
        if not m:
            return None
        return self.idx[self._b[:m].astype(np.int64)], self._o[:m].copy(), self._t[:m].copy()

    def drop(self, b):
        off = C.c_uint64(0)
        self.check(self.lib.krk_window_sched_drop(self.h, self.sub[int(b)], C.byref(off)))
        return off.value

    def close(self):
        if self.h.value:
            self.lib.krk_window_sched_free(self.h)
            self.h = C.c_void_p()


class TailPolicy:
    """Which chains the host threads take, and when (shared by the run and its model).
    A chain is a candidate while it has more bytes left than the window after the queued one
    would give it; candidates go longest-remaining first.  Waiting (not yet admitted) blobs
    are candidates too, with all their bytes left."""

    def __init__(self, lens, threads):
        self.L = np.asarray(lens, dtype=np.int64)
        self.H = max(1, int(threads))
        self.pos = np.zeros(self.L.size, dtype=np.int64)  # bytes the windows queued so far
        self.on_gpu = np.ones(self.L.size, dtype=bool)    # not (yet) taken by a host thread

    def initial(self):
        """The chains the threads take whole before the first window (the H longest)."""
        k = min(self.H, self.L.size)
        first = np.argsort(-self.L, kind="stable")[:k]
        self.on_gpu[first] = False
        return [int(b) for b in first]

    def queued(self, blobs, offs, takes):
        self.pos[blobs] = (offs + takes).astype(np.int64)

    def pick(self, n, min_left):
        """Up to n chains for threads about to be free, most bytes left first; min_left: a
        chain the next window would finish anyway stays on the GPU."""
        if n <= 0:
            return []
        left = np.where(self.on_gpu, self.L - self.pos, -1)
        if n < left.size:
            cand = np.argpartition(-left, n)[:n]
        else:
            cand = np.arange(left.size)
        cand = cand[np.argsort(-left[cand], kind="stable")]
        out = [int(b) for b in cand if left[b] > min_left]
        self.on_gpu[out] = False
        return out


def simulate_tail_handoff(lens, W, cap, threads, rates, launch_s=0.0005, max_chunk=0):
    """The tail handoff on the planner's rates, window by window, with the policy the run uses:
    window k lasts its largest chunk over the per-stream rate of its live count's tier plus a
    launch; at the start of window k (the end of k-1) every thread free within TAIL_HORIZON
    windows after window k takes a chain, whose midstate is ready when window k ends.  Returns the
    modelled end (s), the GPU windows' end, the host bytes and the takeovers."""
    L = np.asarray(lens, dtype=np.int64)
    H = max(0, int(threads))  # 0: the windows alone (the GPU-only model)
    h = tail_thread_rate(rates, max(H, 1))
    pol = TailPolicy(L, max(H, 1))
    first = pol.initial() if H else []
    if not H:
        pol.on_gpu[:] = True
    free = [float(L[b]) / h for b in first] + [0.0] * (H - len(first))
    host_bytes = int(L[first].sum()) if H else 0
    takes = 0
    sched = _Sched(L, np.nonzero(pol.on_gpu)[0], W, cap, max_chunk)
    t = 0.0  # end of the previous window = start of this one
    try:
        win = sched.next()
        while win is not None:
            blobs, offs, tk = win
            pol.queued(blobs, offs, tk)
            dur = float(tk.max()) / stream_rate(rates, blobs.size) + launch_s
            end_k = t + dur
            horizon = end_k + TAIL_HORIZON * dur  # later windows modelled like k
            ready = [i for i in range(H) if free[i] <= horizon]
            chosen = pol.pick(len(ready), stream_rate(rates, blobs.size) * dur)
            ready.sort(key=lambda i: free[i])
            for i, b in zip(ready, chosen):
                y = sched.drop(b)
                start = max(free[i], end_k if y else free[i])
                free[i] = start + float(L[b] - y) / h
                host_bytes += int(L[b] - y)
                takes += 1
            t = end_k
            win = sched.next()
    finally:
        sched.close()
    return {"end_s": max([t] + free), "gpu_end_s": t, "host_bytes": host_bytes, "takeovers": takes + len(first),
            "thread_rate_Bps": h}


def _wait_summary(ws):
    """The tail threads' midstate waits: how many, how many found the window already done,
    wait and assignment-to-start percentiles (ms)."""
    if not ws:
        return {"n": 0}
    w = np.array([x[0] for x in ws]) * 1e3
    a = np.array([x[2] for x in ws]) * 1e3
    return {"n": len(ws), "window_already_done": int(sum(x[1] for x in ws)), "over_5ms": int((w > 5).sum()),
            "wait_ms_p50_p90_max": [round(float(np.percentile(w, q)), 2) for q in (50, 90, 100)],
            "since_assigned_ms_p10_p50_p90": [round(float(np.percentile(a, q)), 1) for q in (10, 50, 90)]}


_CRC_UNQUEUED = object()  # a ring slot whose piece's CRC has not been flushed to the device yet


class TailHandoffRun:
    """A windowed batch (the WindowedRun layout: synthetic blobs generated window by window on
    the device, two device windows, one ChunkedBatch) with the tail handoff: `threads` host
    threads steal chains at window boundaries (TailPolicy).  After run(): cb.sums / cb.digests
    hold every blob's piece sums and digest (device); `stats` the run's takeovers and timing.

    Who does what.  The window loop (the calling thread) owns every device call: the
    windows, and the stolen chains' remaining bytes, generated piece by piece (64 MiB) into
    each thread's ring of device slots on the window generator's stream as slots come free
    and copied down, whole, on one copy stream into a pinned twin of the slot; the pieces'
    CRCs are queued into the window stream after each window's step; each window's midstates
    are mirrored to host memory.  The host threads only wait for their pieces' copies and hash
    them (krk_sha256_resume_host), in order, from the chain's midstate.  Queues: a packet that
    cannot start blocks every later packet of its hardware queue, and normal-priority streams
    share four of them (GPU_MAX_HW_QUEUES; 16 or 32 measured slower, profiles/r06): so the
    windows' step and SHA-256 streams are high priority, the CRC launches (144 KiB-LDS
    workgroups, which wait for CUs the window's SHA workgroups leave room on) go only there,
    and the normal queues carry the copies and the generator's launches (no LDS, never
    blocked, waited for by the host)."""

    def __init__(self, D, ids, lens, P, W, threads, cap=None, device=0, max_chunk=TAIL_CHUNK, piece=TAIL_PIECE,
                 ring=TAIL_RING, crc_after_sha=None, from_previous="auto"):
        self.D = D
        self.ids = np.asarray(ids, dtype=np.uint64)
        self.lens = np.asarray(lens, dtype=np.int64)
        self.P = P
        self.W = int(W)
        self.H = max(1, int(threads))
        self.device = device
        self.max_chunk = int(max_chunk)
        self.piece = int(piece)  # a multiple of 64
        assert self.piece > 0 and self.piece % 64 == 0, piece
        n = self.lens.size
        self.cap = window_stream_cap(D, n) if cap is None else int(cap)
        self.rates = D.planner_rates()
        self.h = tail_thread_rate(self.rates, self.H)
        wb = self.W + 16 * max(min(self.cap, n), 1)
        self.bufs = [D.DeviceBuffer(wb), D.DeviceBuffer(wb)]
        self.cb = D.ChunkedBatch(self.lens, P)
        self.ring = max(2, int(ring))
        self.tbuf = [[D.DeviceBuffer(self.piece) for _ in range(self.ring)] for _ in range(self.H)]
        self.gen_s, self.run_s, self.sha_s = C.c_void_p(), C.c_void_p(), C.c_void_p()
        D.check(D.lib.krk_stream_create_prio(-1, C.byref(self.run_s)))
        D.check(D.lib.krk_stream_create(C.byref(self.gen_s)))
        D.check(D.lib.krk_stream_create_prio(-1, C.byref(self.sha_s)))
        # every window's midstates, copied down after its step on the window stream (window k
        # into mirror k & 1): a stolen chain's midstate is read there once the window is done
        # (a synchronous copy would queue behind other streams' packets in a shared hardware
        # queue)
        self.state_host = [D.PinnedArray((n, 8), np.uint32, dma_target=True) for _ in range(2)]
        # a window's CRC after its SHA launch, or beside it when the windows are full (every
        # stream the cap allows live: throughput-bound windows, where a serialised CRC costs
        # ~13 %; measured beside / after: 1 GPU 537 / 503, 2 GPUs 615 / 586-613, 4 GPUs
        # 720-740 / 746-762, 8 GPUs 946 / 933-954 GB/s, profiles/r06/c3_tail_crc_placement_ab.jsonl)
        if crc_after_sha is None:
            crc_after_sha = min(self.cap, n) < window_stream_cap(D, 1 << 62)  # the device's cap
        self.crc_after_sha = bool(crc_after_sha)
        # "auto": a thread predicted free before the queued window ends takes its chain from the
        # previous window's midstate; "always" / "never": every takeover does / none does (tests)
        assert from_previous in ("auto", "always", "never"), from_previous
        self.from_previous = from_previous
        # the loop copies each generated piece down, whole, on one stream into a pinned twin of
        # its slot (an event a slot); the threads only hash host memory
        self.copy_s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(self.copy_s)))
        # the stolen chains' pieces are generated on a stream of their own (the loop waits for
        # them), the windows' bytes on gen_s behind an event the loop polls while it keeps the
        # threads' rings full (a blocking wait there left the rings unserviced for most of each
        # window: 10.5 of 12.5 s on the 8-GPU shard, 19.2 of 21.7 at N=1)
        self.piece_s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(self.piece_s)))
        self.gen_ev = []
        for _ in range(2):
            e = C.c_void_p()
            D.check(D.lib.krk_event_create_polling(C.byref(e)))
            self.gen_ev.append(e)
        self.hbuf = [[D.PinnedArray((self.piece,), np.uint8, dma_target=True) for _ in range(self.ring)]
                     for _ in range(self.H)]
        self.slot_ev = []
        for _ in range(self.H):
            row = []
            for _ in range(self.ring):
                e = C.c_void_p()
                D.check(D.lib.krk_event_create_polling(C.byref(e)))
                row.append(e)
            self.slot_ev.append(row)
        # every twin written once by DMA before the run (a page's first device write runs at
        # about half the rate: 30 vs 56 GB/s measured), then the twins' copy rate, a record
        # beside the run's copy waits
        import time
        for _ in range(2):
            t0 = time.perf_counter()
            for i in range(self.H):
                for k in range(self.ring):
                    D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(self.hbuf[i][k].ptr),
                                                       C.c_void_p(self.tbuf[i][k].ptr), self.piece, self.copy_s))
            D.check(D.lib.krk_stream_sync(self.copy_s))
            self.twin_GBps = self.H * self.ring * self.piece / (time.perf_counter() - t0) / 1e9
        self.stats = {}

    # ---- the host threads: copy and hash
    def _job(self, i, b, y, win, h0, dig):
        """Chain b from byte y: its pieces as the loop generates them into this thread's ring,
        SHA-256 continued from `h0` (a midstate the loop read at hand-over), else from the
        midstate window `win` left (mirrored to host memory; the loop announces each window's
        end in _win_done, so a worker makes no HIP call to learn it), or from the IV when
        y == 0."""
        D = self.D
        L = int(self.lens[b])
        pieces = self._pieces(y, L)
        nch = len(pieces)
        ph = self._phase[i]
        clk = self._clock
        h = _IV.copy()
        if h0 is not None:
            h = h0
        elif y:
            tw = clk()
            with self._cv:
                done = self._win_done >= win
                while self._win_done < win and not self._abort:  # the window that last advanced b
                    self._cv.wait()
                if self._abort:
                    return
            h = self.state_host[win & 1].a[b].copy()  # copied down before that window's event
            dt = clk() - tw
            ph["midstate"] += dt
            self._mwaits[i].append((dt, done, tw - self._t_assigned.get((i, b), tw)))
        out = np.zeros(32, dtype=np.uint8)
        for c in range(nch):
            t1 = clk()
            with self._cv:  # the next piece of this thread, generated by the loop
                while not self._ready[i] and not self._abort:
                    self._cv.wait()
                if self._abort:
                    return
                k, pb, po, pm = self._ready[i].pop(0)
            assert pb == b and (po, pm) == pieces[c], (pb, po, pm, b, y, c)
            t2 = clk()
            if pm:
                D.check(D.lib.krk_event_sync(self.slot_ev[i][k]))  # the loop's copy of the piece
            ph["copy_wait"] += clk() - t2
            D.check(D.lib.krk_sha256_resume_host(h.ctypes.data_as(C.POINTER(C.c_uint32)), po,
                                                 C.c_void_p(self.hbuf[i][k].ptr), pm, int(c + 1 == nch),
                                                 out.ctypes.data_as(C.POINTER(C.c_uint8))))
            t3 = clk()
            ph["device"] += t2 - t1
            ph["hash"] += t3 - t2
            with self._cv:
                self._slot_used[i][k] = False  # copied down: the loop may refill it once its CRC ran
                self._left[i] -= pm
                self._t_last[i] = t3
                self._done_bytes[i] += pm
                self._cv.notify_all()
        dig[b] = out

    def _worker(self, i, err, dig):
        import time
        try:
            self.D.set_device(self.device)
            w, hh = C.c_double(), C.c_double()
            self.D.check(self.D.lib.krk_sha256_resume_stats(C.byref(w), C.byref(hh)))
            h0 = hh.value  # this thread's SHA-NI seconds so far
            while True:
                with self._cv:
                    while not self._jobs[i] and not self._done and not self._abort:
                        self._cv.wait()
                    if not self._jobs[i] or self._abort:
                        break
                    b, y, win, hm = self._jobs[i][0]
                t0 = time.perf_counter()
                self._job(i, b, y, win, hm, dig)
                with self._cv:
                    self._jobs[i].pop(0)
                    self._busy_s[i] += time.perf_counter() - t0
                    self._cv.notify_all()
            self.D.check(self.D.lib.krk_sha256_resume_stats(C.byref(w), C.byref(hh)))
            self._phase[i]["sha"] = hh.value - h0
        except BaseException as e:  # re-raised on the caller's thread
            err.append(e)
            with self._cv:
                self._abort = True
                self._cv.notify_all()
        finally:
            with self._cv:
                self._alive -= 1
                self._cv.notify_all()

    def _free_at(self, i, now):
        """When thread i is expected to be done with its queued chains, at the rate its pieces
        have been copied and hashed so far (not counting its waits for midstates: a thread
        predicted late gets its next chain late and then waits for it)."""
        t = self._phase[i]["hash"]
        rate = self._done_bytes[i] / t if t > 0.3 else self.h
        return (self._t_last[i] if self._jobs[i] else now) + max(0, self._left[i]) / max(rate, 1e6)

    # ---- the loop's side: generate pieces into free slots, queue their CRCs
    def _assign(self, i, b, y, win, h0=None, crc_from=None):
        """Chain b from byte y (its midstate after window `win`, or h0) becomes thread i's
        next job (caller holds the lock).  Its pieces' CRCs cover bytes from crc_from (y
        unless a window already summed [y, crc_from))."""
        self._jobs[i].append((b, y, win, h0))
        self._t_assigned[(i, b)] = self._clock()
        L = int(self.lens[b])
        cf = y if crc_from is None else int(crc_from)
        # the first piece small (a thread starts hashing after one short copy, not behind a
        # burst of whole-piece copies at a window boundary), the rest whole pieces
        for o, m in self._pieces(y, L):
            self._to_gen[i].append((b, o, m, min(m, max(0, cf - o))))
        self._left[i] += L - y

    def _pieces(self, y, L):
        """A chain's bytes [y, L) as the pieces its thread hashes: a short first one, then
        whole pieces; one empty piece when y == L."""
        out, o = [], y
        while True:
            m = min(TAIL_FIRST_PIECE if o == y else self.piece, self.piece, L - o)
            out.append((o, m))
            o += m
            if o >= L:
                return out

    def _service(self):
        """Every free ring slot (copied down, its CRC queued and done) refilled with its thread's next
        piece: generated on the generator stream, waited for, handed to the thread; their CRCs
        go with the next flush.  Returns the pieces generated."""
        D = self.D
        gen = []
        with self._cv:
            for i in range(self.H):
                while self._to_gen[i]:
                    k = self._next_slot[i]
                    if self._slot_used[i][k]:
                        break
                    ev = self._slot_crc[i][k]
                    if ev is _CRC_UNQUEUED:  # its piece's CRC is not even queued yet
                        break
                    if ev is not None:
                        done = C.c_int(0)
                        D.check(D.lib.krk_event_query(ev, C.byref(done)))
                        if not done.value:
                            break
                        self._slot_crc[i][k] = None
                    b, o, m, c0 = self._to_gen[i].pop(0)
                    self._slot_used[i][k] = True
                    self._slot_crc[i][k] = _CRC_UNQUEUED if m > c0 else None  # until _release
                    self._next_slot[i] = (k + 1) % self.ring
                    gen.append((i, k, b, o, m, c0))
        if not gen:
            return gen
        live = [g for g in gen if g[4] > 0]
        if live:
            ptr = np.array([self.tbuf[i][k].ptr for i, k, _, _, _, _ in live], dtype=np.uint64)
            bl = np.array([g[2] for g in live], dtype=np.int64)
            tg = self._clock()
            D.synth_fill_chunk_arrays(self.ids[bl], ptr, np.array([g[3] for g in live], np.uint64),
                                      np.array([g[4] for g in live], np.uint64), stream=self.piece_s)
            D.check(D.lib.krk_stream_sync(self.piece_s))
            self._gen_wait[0] += self._clock() - tg
            for i, k, _, _, m, _ in live:  # each piece down into its slot's pinned twin, then its event
                D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(self.hbuf[i][k].ptr), C.c_void_p(self.tbuf[i][k].ptr),
                                                   m, self.copy_s))
                D.check(D.lib.krk_event_record(self.slot_ev[i][k], self.copy_s))
        with self._cv:
            for i, k, b, o, m, c0 in gen:
                self._ready[i].append((k, b, o, m))
                if m > c0:  # the CRC of its bytes from c0 on
                    self._pending.append((i, k, b, o + c0, m - c0, c0))
            self._cv.notify_all()
        self._tail_pieces += len(gen)
        return gen

    def _flush_crcs(self, stream):
        """Queue on `stream` the CRCs of the pieces generated since the last flush; returns
        them (their slots are held until the event recorded after this)."""
        D = self.D
        with self._cv:
            take, self._pending = self._pending, []
        if not take:
            return take
        ptr = np.array([self.tbuf[i][k].ptr + c0 for i, k, _, _, _, c0 in take], dtype=np.uint64)
        bl = np.array([t[2] for t in take], dtype=np.int64)
        arr = D.chunk_array(ptr, np.array([t[3] for t in take], np.uint64), np.array([t[4] for t in take], np.uint64),
                            self.cb.lengths[bl], self.cb.piece_lengths[bl], self.cb.sums_off[bl],
                            bl.astype(np.uint64))
        D.check(D.lib.krk_chunks_crc_dev(arr.ctypes.data_as(C.POINTER(D.krk_chunk)), len(take), self.cb.sums.ptr,
                                         stream))
        return take

    def _release(self, take, ev):
        with self._cv:
            for t in take:
                self._slot_crc[t[0]][t[1]] = ev

    def _wait_window(self, ev):
        """Until window event `ev` completes, keep the threads' rings full."""
        D = self.D
        done = C.c_int(0)
        while True:
            D.check(D.lib.krk_event_query(ev, C.byref(done)))
            if done.value:
                return
            if not self._service():
                with self._cv:
                    self._cv.wait(0.002)

    def run(self):
        import threading
        import time
        D = self.D
        n = self.lens.size
        self._clock = time.perf_counter
        self._mu = threading.Lock()
        self._cv = threading.Condition(self._mu)
        H, R = self.H, self.ring
        self._jobs = [[] for _ in range(H)]
        self._to_gen = [[] for _ in range(H)]   # pieces the loop still has to generate, in order
        self._ready = [[] for _ in range(H)]    # generated pieces a thread may copy and hash, in order
        self._slot_used = [[False] * R for _ in range(H)]
        self._slot_crc = [[None] * R for _ in range(H)]  # the event after the slot's last CRC
        self._next_slot = [0] * H
        self._pending = []
        self._left = [0] * H
        self._t_last = [0.0] * H
        self._busy_s = [0.0] * H
        self._done_bytes = [0] * H
        self._phase = [{"midstate": 0.0, "device": 0.0, "hash": 0.0, "copy_wait": 0.0} for _ in range(H)]
        self._mwaits = [[] for _ in range(H)]  # (wait s, event already done, s since assignment)
        self._t_assigned = {}
        self._tail_pieces = 0
        self._gen_wait = [0.0, 0.0]  # the loop's seconds generating: tail pieces, windows
        self._done = self._abort = False
        self._win_done = -1  # the last window the loop has seen end
        self._alive = H
        dig = np.zeros((n, 32), dtype=np.uint8)
        err = []
        pol = TailPolicy(self.lens, H)
        host_blobs = set()
        host_bytes = 0
        t0 = self._clock()
        with self._cv:
            for i, b in enumerate(pol.initial()):
                self._assign(i, b, 0, None)
                self._t_last[i] = t0
                host_blobs.add(b)
                host_bytes += int(self.lens[b])
        workers = [threading.Thread(target=self._worker, args=(i, err, dig), name=f"krk-tail-{i}")
                   for i in range(H)]
        for w in workers:
            w.start()
        sched = _Sched(self.lens, np.nonzero(pol.on_gpu)[0], self.W, self.cap, self.max_chunk)
        evs = []

        def new_event():
            e = C.c_void_p()
            D.check(D.lib.krk_event_create(C.byref(e)))
            evs.append(e)
            return e

        takes, resumed, early, wait_win_s = 0, 0, 0, 0.0
        scale = 1.0  # measured / modelled window time (EMA)
        gpu_end = 0.0
        wev = []  # the windows' events
        try:
            self._service()
            win = sched.next()
            k = 0
            items = self._items(win, 0) if win is not None else None
            if items is not None:
                self._gen(items, 0)
            t_prev_end = self._clock()
            last_model = 1.0
            while win is not None and not err:
                blobs, offs, tk = win
                tg = self._clock()
                self._wait_window(self.gen_ev[k & 1])  # window k's bytes
                self._gen_wait[1] += self._clock() - tg
                pol.queued(blobs, offs, tk)
                self.cb.step_arrays(items[0], items[1], items[2], items[3], stream=self.run_s, sha_stream=self.sha_s,
                                    crc_after_sha=self.crc_after_sha)
                take = self._flush_crcs(self.run_s)
                D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(self.state_host[k & 1].ptr), C.c_void_p(self.cb.state.ptr),
                                                   32 * n, self.run_s))
                ev = new_event()
                D.check(D.lib.krk_event_record(ev, self.run_s))
                wev.append(ev)
                self._release(take, ev)
                model = float(tk.max()) / stream_rate(self.rates, blobs.size) + 0.0005
                if k:
                    tw = self._clock()
                    self._wait_window(wev[k - 1])
                    with self._cv:
                        self._win_done = k - 1
                        self._cv.notify_all()
                    now = self._clock()
                    wait_win_s += now - tw
                    scale = 0.7 * scale + 0.3 * max(0.2, min(5.0, (now - t_prev_end) / max(last_model, 1e-6)))
                    t_prev_end = now
                now = self._clock()
                last_model = model
                end_k = now + model * scale
                horizon = end_k + TAIL_HORIZON * model * scale  # later windows modelled like k
                with self._cv:  # threads with at most their current chain, free before k+1 ends
                    ready = [i for i in range(H) if len(self._jobs[i]) <= 1 and self._free_at(i, now) <= horizon]
                    ready.sort(key=lambda i: self._free_at(i, now))
                    before_k = {i: (self.from_previous == "always" or
                                    (self.from_previous == "auto" and self._free_at(i, now) < end_k)) for i in ready}
                chosen = pol.pick(len(ready), stream_rate(self.rates, blobs.size) * model)
                with self._cv:
                    for i, b in zip(ready, chosen):
                        y = sched.drop(b)
                        if not self._jobs[i]:
                            self._t_last[i] = now
                        if y and before_k[i]:
                            # free before window k ends: start from the midstate window k-1 left
                            # (done, mirrored, read now), hashing window k's chunk of b again on
                            # the host; the window keeps that chunk's CRC, the thread's pieces
                            # sum from y on
                            j = np.flatnonzero(blobs == b)
                            yp = int(offs[j[0]]) if j.size else y
                            h0 = self.state_host[(k - 1) & 1].a[b].copy() if yp else _IV.copy()
                            self._assign(i, b, yp, -1, h0=h0, crc_from=y)
                            early += 1
                        else:
                            yp = y
                            self._assign(i, b, y, k if y else -1)
                        host_blobs.add(b)
                        host_bytes += int(self.lens[b]) - yp
                        takes += 1
                        resumed += yp > 0
                    self._cv.notify_all()
                self._service()
                win = sched.next()
                k += 1
                if win is not None:
                    items = self._items(win, k)
                    self._gen(items, k)
            if wev:
                self._wait_window(wev[-1])
                with self._cv:
                    self._win_done = len(wev) - 1
                    self._cv.notify_all()
            gpu_end = self._clock() - t0
            with self._cv:
                self._done = True
                self._cv.notify_all()
            # the windows are done: keep the rings full and the pieces' CRCs flushed
            while not err:
                with self._cv:
                    if self._alive == 0:
                        break
                self._service()
                take = self._flush_crcs(self.run_s)
                if take:
                    ev = new_event()
                    D.check(D.lib.krk_event_record(ev, self.run_s))
                    self._release(take, ev)
                with self._cv:
                    self._cv.wait(0.002)
            take = self._flush_crcs(self.run_s)  # the last pieces (every thread is done)
            if take:
                ev = new_event()
                D.check(D.lib.krk_event_record(ev, self.run_s))
                self._release(take, ev)
        except BaseException:  # the loop failed: the threads must not wait for it
            with self._cv:
                self._abort = True
                self._cv.notify_all()
            raise
        finally:
            with self._cv:
                self._done = True
                if err:
                    self._abort = True
                self._cv.notify_all()
            for w in workers:
                w.join()
            sched.close()
        try:
            if err:
                raise err[0]
            D.check(D.lib.krk_stream_sync(self.run_s))  # the last tail CRCs
            for b in sorted(host_blobs):
                row = np.ascontiguousarray(dig[b])
                D.check(D.lib.krk_memcpy_h2d(C.c_void_p(self.cb.digests.ptr + 32 * int(b)),
                                             row.ctypes.data_as(C.c_void_p), 32))
        finally:
            D.lib.krk_stream_sync(self.run_s)
            for e in evs:
                D.lib.krk_event_destroy(e)
        self.stats = {"windows": len(wev), "gpu_windows_end_s": round(gpu_end, 3),
                      "takeovers": takes, "resumed_from_midstate": resumed, "from_previous_window": early,
                      "host_chains": len(host_blobs),
                      "host_bytes": host_bytes, "tail_pieces": self._tail_pieces,
                      "thread_busy_s": [round(x, 3) for x in self._busy_s],
                      "thread_GBps": [round(self._done_bytes[i] / max(self._busy_s[i], 1e-9) / 1e9, 3)
                                      for i in range(H)],
                      "thread_phases_s": {k: round(sum(p.get(k, 0.0) for p in self._phase), 3)
                                          for k in ("midstate", "device", "hash", "copy_wait", "sha")},
                      "loop_wait_s": round(wait_win_s, 3), "window_time_scale": round(scale, 3),
                      "midstate_waits": _wait_summary([w for ws in self._mwaits for w in ws]),
                      "twin_copy_GBps_before_run": round(self.twin_GBps, 2), "crc_after_sha": self.crc_after_sha,
                      "loop_generate_s": {"tail_pieces": round(self._gen_wait[0], 3),
                                          "windows": round(self._gen_wait[1], 3)}}

    def _items(self, win, k):
        blobs, offs, take = win
        dev = np.zeros(take.size, dtype=np.uint64)
        dev[1:] = np.cumsum((take + np.uint64(15)) // np.uint64(16) * np.uint64(16))[:-1]
        dev += np.uint64(self.bufs[k & 1].ptr)
        return blobs, dev, offs, take

    def _gen(self, items, k):
        """Window k's bytes generated on gen_s; gen_ev[k & 1] marks them done."""
        blobs, dev, offs, take = items
        self.D.synth_fill_chunk_arrays(self.ids[blobs], dev, offs, take, stream=self.gen_s)
        self.D.check(self.D.lib.krk_event_record(self.gen_ev[k & 1], self.gen_s))

    def close(self):
        for s in [self.gen_s, self.run_s, self.sha_s, self.copy_s, self.piece_s]:  # nothing in flight
            if s.value:
                self.D.lib.krk_stream_sync(s)
        for b in self.bufs + [x for ring in self.tbuf for x in ring]:
            b.free()
        self.bufs, self.tbuf, self.hbuf = [], [], []
        for e in [e for row in self.slot_ev for e in row]:
            self.D.lib.krk_event_destroy(e)
        self.slot_ev = []
        for s in [self.gen_s, self.run_s, self.sha_s, self.copy_s, self.piece_s]:
            if s.value:
                self.D.lib.krk_stream_sync(s)
                self.D.lib.krk_stream_destroy(s)
        for e in self.gen_ev:
            self.D.lib.krk_event_destroy(e)
        self.gen_ev = []
        self.gen_s, self.run_s, self.sha_s, self.copy_s, self.piece_s = (C.c_void_p(), C.c_void_p(), C.c_void_p(),
                                                                          C.c_void_p(), C.c_void_p())

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
