"""Diagnose the C3 host-lane windowed mismatch (tests/test_gpu_windowed.py lane2): run the
test's configuration under one of several modes and report every blob whose piece sums
differ from the one-shot device run.

    python tools/lane_diag.py MODE
MODE: base | seq (lane first, then the windows) | nocrc (the lane skips its CRCs) |
      nohash (the lane skips its SHA-256) | nolane (no lane, same window plan minus the
      lane blobs is not possible, so: the plain windowed run)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kraken_amd import device as D  # noqa: E402
from kraken_amd.windowed import WindowedRun, c3_lengths  # noqa: E402

N, SCALE, P = 1500, 16, 4 << 20


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "base"
    D.set_device(0)
    lens = c3_lengths(N, scale=SCALE)
    ids = [(2 << 40) + i for i in range(N)]
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    sums1 = out.sums.to_host(np.uint32, arena.total_pieces)
    dg1 = out.digests.to_host(np.uint8, 32 * N).reshape(-1, 32)
    offs1, counts1 = arena.sums_off.copy(), arena.n_pieces.copy()
    del arena, out
    wr = WindowedRun(D, ids, lens, P, 1 << 30, cap=200, host_lane=None if mode == "nolane" else (100, 8))
    if mode == "nocrc":
        orig = D.piece_sums_dev_arrays
        D.piece_sums_dev_arrays = lambda *a, **k: None
    if mode == "nohash":
        D.sha256_dev_on_host = lambda ptrs, lens, threads=0, stream=None: np.zeros((len(ptrs), 32), np.uint8)
    t0 = time.perf_counter()
    if mode == "seq":
        err = []
        wr._lane(err)
        assert not err, err
        wr._run_windows()
        for i in wr.lane_blobs:
            import ctypes as C
            row = np.ascontiguousarray(wr.lane_digests[i])
            D.check(D.lib.krk_memcpy_h2d(C.c_void_p(wr.cb.digests.ptr + 32 * int(i)), row.ctypes.data_as(C.c_void_p), 32))
    else:
        wr.run()
    el = time.perf_counter() - t0
    cb = wr.cb
    dg = cb.digests.to_host(np.uint8, 32 * N).reshape(-1, 32)
    sums = cb.sums.to_host(np.uint32, cb.total_pieces)
    lane = set(int(i) for i in wr.lane_blobs)
    bad = []
    for i in range(N):
        a, b = int(cb.sums_off[i]), int(offs1[i])
        x, y = sums[a:a + int(counts1[i])], sums1[b:b + int(counts1[i])]
        if not np.array_equal(x, y):
            first = int(np.flatnonzero(x != y)[0])
            bad.append((i, "lane" if i in lane else "win", first, int(counts1[i]), int((x == 0).sum())))
    dbad = [i for i in range(N) if not np.array_equal(dg[i], dg1[i]) and (mode != "nohash" or i not in lane)]
    # the windows each blob's chunks ran in
    last = {}
    for k, (blobs, offs, take) in enumerate(wr.wins):
        for b, o, t in zip(blobs, offs, take):
            last.setdefault(int(b), []).append((k, int(o), int(t)))
    print(f"mode={mode} run {el:.2f} s, windows {len(wr.wins)}, lane blobs {len(lane)}, "
          f"sum mismatches {len(bad)}, digest mismatches {len(dbad)}")
    for i, kind, first, n, zeros in bad[:20]:
        ch = last.get(i, [])
        tail = [(k, o, t) for k, o, t in ch if o + t > first * P]
        print(f"  blob {i} ({kind}, len {lens[i]}): first bad piece {first} of {n}, zero pieces {zeros}; "
              f"chunks from the first bad piece: {tail[:6]}{' ...' if len(tail) > 6 else ''} of {len(ch)}")
    wr.close()


if __name__ == "__main__":
    main()
