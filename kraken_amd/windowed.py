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
    """Windows: [(blob indices, offsets, chunk lengths)].  Every live blob advances by
    the same 64-multiple chunk per window (about W bytes a window).  Admission: at most
    `cap` blobs are live, admitted longest first, so the longest chain starts in window 0
    and every window stays on a multi-lane SHA plan (eight lanes a stream up to 16 x CUs
    live streams, two up to 64 x CUs; a launch of more streams falls back to one lane per
    stream, ~0.7x per stream); a finished blob's slot goes to the
    next-longest waiting blob."""
    L = np.asarray(lens, dtype=np.uint64)
    n = L.size
    cap = max(1, min(int(cap), n)) if n else 1
    queue = list(np.argsort(-L.astype(np.int64), kind="stable"))
    wins, pos = [], np.zeros(n, dtype=np.uint64)
    live = np.asarray(sorted(queue[:cap]), dtype=np.int64)
    queue = queue[cap:]
    while live.size:
        c = max(64, (W // live.size) // 64 * 64)
        take = np.minimum(np.uint64(c), L[live] - pos[live])
        wins.append((live, pos[live].copy(), take))
        pos[live] += take
        live = live[pos[live] < L[live]]
        if queue and live.size < cap:
            k = cap - live.size
            live = np.sort(np.concatenate([live, np.asarray(queue[:k], dtype=np.int64)]))
            queue = queue[k:]
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
    multiple of the two-pair workgroup's 64 streams).  At the full two-lane count
    (64 x CUs) every CU holds a 128 KiB SHA workgroup and the window's piece-CRC launch
    (144 KiB workgroups) waits for the SHA launch to end; with an eighth of the CUs left
    free it runs inside it, and the chain of the longest blob -- not the live count --
    still sets the run time.  C3 on one MI355X (bench --live-cap): 16,384 live 494 GB/s,
    15,360 522, 14,336 524, 13,824 523, 13,312 522, 12,288 509 (profiles/r02/c3_live_cap.jsonl)."""
    full = two_lane_stream_cap(D, 1 << 30) if n else 1
    cap = max(64, (full * 7 // 8) // 64 * 64)
    return max(1, min(n, cap))


class WindowedRun:
    """One batch of synthetic blobs (ids, lens, piece length P) streamed through two
    device windows of W bytes: window k+1 is generated on `gen` while window k's
    kernels run on `run`.  After run(): cb.sums / cb.digests hold every blob's piece
    sums and digest (device)."""

    def __init__(self, D, ids, lens, P, W, cap=None):
        self.D = D
        self.ids = np.asarray(ids, dtype=np.uint64)
        self.lens = list(lens)
        self.P = P
        self.W = int(W)
        n = len(self.lens)
        self.cap = window_stream_cap(D, n) if cap is None else int(cap)
        self.wins = window_plan(self.lens, self.W, self.cap)
        self.bufs = [D.DeviceBuffer(self.W + 16 * n), D.DeviceBuffer(self.W + 16 * n)]
        self.cb = D.ChunkedBatch(self.lens, P)
        self.gen_s, self.run_s = C.c_void_p(), C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(self.gen_s)))
        D.check(D.lib.krk_stream_create(C.byref(self.run_s)))

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

    def run(self):
        """Window k's kernels are queued before the host waits for window k-1's (an
        event after each window), so the device goes from one window to the next with
        no host round trip; window k+1 is generated into k-1's buffer once k-1 is done."""
        D = self.D
        cur = self._items(0)
        self._gen(cur)
        evs = [C.c_void_p(), C.c_void_p()]
        for e in evs:
            D.check(D.lib.krk_event_create(C.byref(e)))
        try:
            for k in range(len(self.wins)):
                self.cb.step_arrays(cur[0], cur[1], cur[2], cur[3], stream=self.run_s)
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
        for b in self.bufs:
            b.free()
        self.bufs = []
        for s in (self.gen_s, self.run_s):
            if s.value:
                self.D.lib.krk_stream_destroy(s)
        self.gen_s = self.run_s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
