"""Re-entrancy of the C ABI (SURVEY.md §8(b) "Threading": HTTP handlers, the
blobrefresh worker pool and P2P dispatch call NewMetaInfo / Digester /
PieceHash / Locations from many goroutines at once).  Eight host threads call
the host-buffer entry points concurrently (ctypes drops the GIL for the call);
every result must equal the single-threaded reference."""
import hashlib
import io
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from kraken_amd import agentstorage, core, hrw
from kraken_amd import device as D

pytestmark = pytest.mark.gpu


def _work(seed: int):
    D.set_device(0)  # per calling thread (krk_set_device)
    rng = np.random.default_rng(seed)
    out = []
    # Digester streaming writes
    data = rng.integers(0, 256, int(rng.integers(1, 3 << 20)), dtype=np.uint8).tobytes()
    d = core.NewDigester()
    for i in range(0, len(data), 700_001):
        d._write(data[i:i + 700_001])
    out.append(d.Digest().Hex() == hashlib.sha256(data).hexdigest())
    # NewMetaInfo over a reader (piece stream) vs zlib per piece
    P = int(rng.choice([3, 4096, 65536, 1 << 20]))
    small = data[:200_000]
    mi = core.NewMetaInfo(core.NewDigester().FromBytes(small), io.BytesIO(small), P)
    ref = [zlib.crc32(small[i:i + P]) for i in range(0, len(small), P)]
    out.append(mi.PieceSums().tolist() == ref)
    # PieceHash
    h = core.PieceHash()
    h.Write(data[:12345])
    out.append(h.Sum32() == zlib.crc32(data[:12345]))
    # batched host metainfo + digest
    blobs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, 1 << 20, 6)]
    sums, dg = D.metainfo_digest_host(blobs, 1 << 18)
    for b, s, g in zip(blobs, sums, dg):
        out.append(bytes(g) == hashlib.sha256(b.tobytes()).digest())
        out.append(s.tolist() == [zlib.crc32(b[i:i + (1 << 18)].tobytes()) for i in range(0, b.size, 1 << 18)])
    # agent piece verification
    pieces = [data[i:i + 5000] for i in range(0, 50_000, 5000)]
    out.append(bool(agentstorage.verify_pieces(pieces, [zlib.crc32(p) for p in pieces]).all()))
    # HRW ordering
    rh = hrw.NewRendezvousHash()
    for k in range(5):
        rh.AddNode(f"origin-{k:03d}.kraken.test:15002", 100)
    keys = [rng.bytes(2).hex() for _ in range(50)]
    out.append([o.tolist() for o in rh.GetOrderedNodesBatch(keys, 5)])
    return out


def test_concurrent_callers_match_serial(gpu):
    serial = [_work(s) for s in range(8)]
    for r in serial:
        assert all(x is True for x in r[:-1])
    with ThreadPoolExecutor(8) as ex:
        for rounds in range(2):
            par = list(ex.map(_work, range(8)))
            assert par == serial


def test_init_shutdown_reinit(gpu, orc):
    """krk_init / krk_shutdown: contexts (and the kept staging windows) are freed and
    re-created lazily; results are unchanged across the cycle.  A mask bit past the
    visible devices is KRK_ENODEV."""
    import numpy as np
    from kraken_amd import device as Dv
    from kraken_amd._capi import KRK_ENODEV, lib as L
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (1, 4097, (2 << 20) + 3)]
    pls = [4096, 4096, 1 << 20]
    Dv.init(0)
    first = Dv.metainfo_digest_host(data, pls)
    Dv.shutdown()
    again = Dv.metainfo_digest_host(data, pls)  # lazily re-created context
    Dv.shutdown()
    Dv.init(1)
    third = Dv.metainfo_digest_host(data, pls)
    for r in (first, again, third):
        for i, d in enumerate(data):
            assert np.array_equal(r[0][i], orc.calc_piece_sums(d, pls[i])[1])
            assert bytes(r[1][i]) == __import__("hashlib").sha256(d.tobytes()).digest()
    assert L.krk_init(1 << 63) == KRK_ENODEV


def test_uploads_behind_a_long_kernel_on_many_streams(gpu):
    """upload()'s pinned slots (runtime.hpp UploadRing) when one stream's copies wait: a
    window step whose CRC pack copy waits (on another library stream, behind an event) for
    a ~0.8 s SHA-256 kernel, while 40 threads on streams of their own (more than the 32
    rings: some share) upload piece-sum packs, then destroy their streams.  Every result
    must equal the one-shot device run of the same bytes: a slot rewritten before its copy
    ran would hand a launch another call's work items (piece sums XOR'd twice or missed)."""
    import ctypes as C
    import threading
    P = 1 << 20
    long_arena = D.BlobArena([48 << 20], P, blob_ids=[901])
    long_out = D.BatchOutputs(long_arena)
    # the window step's blobs and every thread's blobs, with their one-shot results
    win_lens = [(k * 977_777) % (3 << 20) + 1 for k in range(1, 41)]
    win = D.BlobArena(win_lens, P, blob_ids=range(1000, 1040))
    wref = D.BatchOutputs(win)
    D.metainfo_digest(win, wref)
    thr = [D.BlobArena([(t * 7919 + k * 104_729) % (2 << 20) + 1 for k in range(3)], 1 << 18,
                       blob_ids=[2000 + 3 * t + k for k in range(3)]) for t in range(40)]
    tref = []
    for a in thr:
        o = D.BatchOutputs(a)
        D.piece_sums(a, o)
        tref.append(o)
    D.synchronize()
    wsums = wref.sums.to_host(np.uint32, win.total_pieces)
    wdig = wref.digests.to_host(np.uint8, 32 * len(win_lens))
    trefs = [o.sums.to_host(np.uint32, a.total_pieces) for a, o in zip(thr, tref)]

    s = C.c_void_p()
    D.check(D.lib.krk_stream_create(C.byref(s)))
    cb = D.ChunkedBatch(win_lens, P)
    errs = []

    def worker(t):
        try:
            D.set_device(0)
            st = C.c_void_p()
            D.check(D.lib.krk_stream_create(C.byref(st)))
            out = D.BatchOutputs(thr[t])
            for _ in range(12):
                D.piece_sums(thr[t], out, stream=st)
                D.check(D.lib.krk_stream_sync(st))
                got = out.sums.to_host(np.uint32, thr[t].total_pieces)
                if not np.array_equal(got, trefs[t]):
                    errs.append(f"thread {t}")
            D.lib.krk_stream_destroy(st)
        except Exception as e:  # re-raised below
            errs.append(repr(e))

    try:
        D.sha256(long_arena, long_out, stream=s)  # ~0.8 s on one stream
        ptrs = np.uint64(win.buf.ptr) + win.offsets
        cb.step_arrays(np.arange(len(win_lens)), ptrs, np.zeros(len(win_lens), np.uint64), win.lengths, stream=s)
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(40)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        D.check(D.lib.krk_stream_sync(s))
    finally:
        D.lib.krk_stream_destroy(s)
    assert not errs, errs[:5]
    assert np.array_equal(cb.sums.to_host(np.uint32, cb.total_pieces), wsums)
    assert np.array_equal(cb.digests.to_host(np.uint8, 32 * len(win_lens)), wdig)


def test_async_d2h_on_two_streams(gpu):
    """krk_memcpy_d2h_async (the C4 back-to-back steps): copies queued on two library streams
    behind piece-sum launches land in pinned arrays once each stream is synchronised, and
    equal the synchronous copy."""
    import ctypes as C
    arena = D.BlobArena([(3 << 20) + 5, 1 << 20, 77], 1 << 18, blob_ids=[9, 10, 11])
    outs = [D.BatchOutputs(arena), D.BatchOutputs(arena)]
    pins = [D.PinnedArray((arena.total_pieces,), np.uint32) for _ in range(2)]
    streams = [C.c_void_p(), C.c_void_p()]
    for st in streams:
        D.check(D.lib.krk_stream_create(C.byref(st)))
    try:
        for k in range(2):
            D.piece_sums(arena, outs[k], stream=streams[k])
            pins[k].fill_from_async(outs[k].sums, streams[k])
        for st in streams:
            D.check(D.lib.krk_stream_sync(st))
        want = outs[0].sums.to_host(np.uint32, arena.total_pieces)
        assert want.any()
        for p in pins:
            assert np.array_equal(p.a, want)
    finally:
        for st in streams:
            D.lib.krk_stream_destroy(st)


def test_streams_come_and_go(gpu):
    """Library streams created, used and destroyed one after another (what every
    WindowedRun does): the library's events last recorded on a destroyed stream (upload
    slots, idle scratch blocks) are replaced before it goes (krk_stream_destroy), so later
    calls on other streams -- and a kernel launch on the default stream -- neither wait on
    nor report the dead stream ("operation not permitted when stream is capturing" once)."""
    import ctypes as C
    from kraken_amd import hrw
    arena = D.BlobArena([(1 << 20) + 17, 333, 5 << 18], 1 << 18, blob_ids=[41, 42, 43])
    ref = D.BatchOutputs(arena)
    D.piece_sums(arena, ref)
    D.synchronize()
    want = ref.sums.to_host(np.uint32, arena.total_pieces)
    out = D.BatchOutputs(arena)
    for k in range(60):
        st = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(st)) if k % 2 else D.lib.krk_stream_create_prio(-1, C.byref(st)))
        D.piece_sums(arena, out, stream=st)
        D.check(D.lib.krk_stream_destroy(st))  # no sync first: destroy waits for the stream's work
        assert np.array_equal(out.sums.to_host(np.uint32, arena.total_pieces), want), k
        D.piece_sums(arena, out)  # the default stream, reusing the dead stream's blocks
        D.synchronize()
        assert np.array_equal(out.sums.to_host(np.uint32, arena.total_pieces), want), k
    rh = hrw.NewRendezvousHash()
    for i in range(4):
        rh.AddNode(f"n{i}", 100)
    assert len(rh.GetOrderedNodes("abcd", 3)) == 3  # a launch after all of it reports no stale error
