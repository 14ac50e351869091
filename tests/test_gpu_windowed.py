"""Config C3's windowed path (kraken_amd.windowed, the machinery bench.py's C3 line
runs): blobs larger in total than HBM advance chunk by chunk through two device
windows -- SHA-256 from per-blob midstates, piece CRCs XOR-accumulated by byte range
(krk_metainfo_digest_chunks_dev) -- with the next window generated on its own stream
and blobs admitted longest first under the live cap.  A scaled C3: 1,500 blobs drawn
from the C3 length law with every length divided by 16 (6.5-67 MB,
byte-granular, so nearly every blob ends in a partial piece), 4 MiB pieces.  Every
blob is checked against the one-shot device path, sampled blobs against hashlib /
the oracle."""
import hashlib

import numpy as np
import pytest

from kraken_amd import device as D
from kraken_amd.windowed import WindowedRun, c3_lengths, window_plan

pytestmark = pytest.mark.gpu

N, SCALE, P = 1500, 16, 4 << 20


@pytest.fixture(scope="module")
def one_shot(gpu):
    lens = c3_lengths(N, scale=SCALE)
    ids = [(2 << 40) + i for i in range(N)]
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    dg = out.digests.to_host(np.uint8, 32 * N).reshape(-1, 32)
    sums = out.sums.to_host(np.uint32, arena.total_pieces)
    offs, counts = arena.sums_off.copy(), arena.n_pieces.copy()
    del arena, out
    return lens, ids, dg, sums, offs, counts


@pytest.mark.parametrize("window_gib,cap,lane", [(4, None, None), (1, 200, None), (1, 200, (100, 8))])
def test_windowed_c3_matches_one_shot_and_oracle(one_shot, orc, window_gib, cap, lane):
    """lane=(K, T): the K longest blobs go through the host lane (generated into their
    own device buffer T at a time, piece CRCs on the GPU, SHA-256 on T host threads
    reading HBM) while the windows run the rest; the last group is partial (100 = 12 x 8
    + 4) and every result must still match."""
    lens, ids, dg1, sums1, offs1, counts1 = one_shot
    wr = WindowedRun(D, ids, lens, P, window_gib << 30, cap=cap, host_lane=lane)
    if lane:
        assert len(wr.lane_blobs) == lane[0] and len(wr.lane_groups) == 13
        assert not set(wr.lane_blobs) & set(np.concatenate([w[0] for w in wr.wins]).tolist())
        assert min(lens[i] for i in wr.lane_blobs) >= max(lens[int(i)] for w in wr.wins for i in w[0])
    if cap is None:
        assert wr.cap >= N  # production admission: the two-lane cap exceeds this batch
    else:
        live = max(len(w[0]) for w in wr.wins)
        assert live <= cap < N and len(wr.wins) > (40 if lane else 50)
    wr.run()
    cb = wr.cb
    dg = cb.digests.to_host(np.uint8, 32 * N).reshape(-1, 32)
    sums = cb.sums.to_host(np.uint32, cb.total_pieces)
    wr.close()
    assert np.array_equal(dg, dg1)
    for i in range(N):
        a, b = int(cb.sums_off[i]), int(offs1[i])
        assert np.array_equal(sums[a:a + int(counts1[i])], sums1[b:b + int(counts1[i])]), i
    L = np.asarray(lens)
    partial = int(np.flatnonzero(L % P)[0])
    for i in sorted({int(L.argmin()), int(L.argmax()), partial, 7, 777}):
        data = orc.synth(ids[i], lens[i])
        assert bytes(dg[i]) == hashlib.sha256(data.tobytes()).digest(), i
        a = int(cb.sums_off[i])
        assert np.array_equal(sums[a:a + int(counts1[i])], orc.calc_piece_sums(data, P)[1]), i


def test_window_plan_covers_c3_law_once():
    """The plan itself at the production scale of one rank's C3 shard (host only)."""
    lens = c3_lengths(2500)
    wins = window_plan(lens, 48 << 30, 8192)
    pos = np.zeros(len(lens), dtype=np.uint64)
    for blobs, offs, take in wins:
        assert np.array_equal(pos[blobs], offs)
        assert ((take % 64 == 0) | (offs + take == np.asarray(lens, dtype=np.uint64)[blobs])).all()
        pos[blobs] += take
    assert np.array_equal(pos, np.asarray(lens, dtype=np.uint64))


@pytest.mark.parametrize("cap,threads,piece,ring,prev", [(None, 3, 64 << 20, 8, "auto"), (200, 4, 64 << 20, 8, "never"),
                                                         (None, 5, 1 << 20, 8, "always"), (None, 5, 1 << 20, 2, "auto"),
                                                         (200, 4, 64 << 20, 8, "always")])
def test_tail_handoff_matches_one_shot_and_oracle(one_shot, orc, cap, threads, piece, ring, prev):
    """the windowed batch with the tail handoff (windowed.TailHandoffRun):
    host threads start on the longest chains whole, then steal the chains with the most bytes
    left at window boundaries -- live chains from the midstate the windows left in HBM, and
    (cap=200) blobs still waiting for admission from the IV -- while their remaining piece
    CRCs run on the GPU beside the windows'.  1 MiB window chunks: hundreds of windows and
    takeovers.  piece=1 MiB: a thread's chain spans many device pieces, so its ring wraps
    inside one chain and one window's CRC flush carries several pieces of one blob; ring=2
    wraps inside one window wait, where a slot a thread has copied down may not be refilled
    before its piece's CRC is queued (a round-6 failure: right digests, wrong sums).
    prev="always": every chain changes hands from the midstate the PREVIOUS window left, the
    thread hashing the queued window's chunk again while the window keeps that chunk's CRC
    (its pieces sum from the window's end on); "never": always from the queued window's.
    Every blob equals the one-shot device path; sampled blobs the oracle."""
    from kraken_amd.windowed import TailHandoffRun
    lens, ids, dg1, sums1, offs1, counts1 = one_shot
    tr = TailHandoffRun(D, ids, lens, P, 200 << 20, threads, cap=cap, max_chunk=1 << 20, piece=piece, ring=ring,
                        from_previous=prev)
    tr.run()
    st = tr.stats
    cb = tr.cb
    dg = cb.digests.to_host(np.uint8, 32 * N).reshape(-1, 32)
    sums = cb.sums.to_host(np.uint32, cb.total_pieces)
    tr.close()
    print(st)
    assert st["takeovers"] > threads and st["resumed_from_midstate"] > 0 and st["windows"] > 50, st
    assert 0 < st["host_bytes"] < int(np.sum(lens)), st
    assert st["tail_pieces"] >= st["host_chains"], st
    if prev == "never":
        assert st["from_previous_window"] == 0, st
    if prev == "always":
        assert st["from_previous_window"] >= st["resumed_from_midstate"] > 0, st
    bad = [i for i in range(N) if bytes(dg[i]) != bytes(dg1[i])]
    assert not bad, (len(bad), bad[:10])
    for i in range(N):
        a, b = int(cb.sums_off[i]), int(offs1[i])
        assert np.array_equal(sums[a:a + int(counts1[i])], sums1[b:b + int(counts1[i])]), i
    L = np.asarray(lens)
    for i in sorted({int(L.argmin()), int(L.argmax()), 7, 777}):
        data = orc.synth(ids[i], lens[i])
        assert bytes(dg[i]) == hashlib.sha256(data.tobytes()).digest(), i
        a = int(cb.sums_off[i])
        assert np.array_equal(sums[a:a + int(counts1[i])], orc.calc_piece_sums(data, P)[1]), i


def test_sha256_resume_from_device_bytes(gpu, orc):
    """krk_sha256_resume_dev_on_host: one chain continued on the calling thread from device
    bytes, in runs of whole blocks then a final run of any length (0, 1, 55, 56, 64, 8 MiB +
    3 ...), equals hashlib over the whole blob."""
    import ctypes as C
    from kraken_amd.windowed import _IV
    for L, cuts in ((0, []), (1, []), (55, []), (64, []), (128, [64]), (130, [64]), ((8 << 20) + 3, [1 << 20, 3 << 20]),
                    ((17 << 20) + 64, [64, (16 << 20) + 64])):
        data = orc.synth(4242 + L, L)
        buf = D.DeviceBuffer(max(L, 1))
        if L:
            buf.from_host(data)
        h = _IV.copy()
        out = np.zeros(32, np.uint8)
        prev = 0
        for c in cuts + [L]:
            D.check(D.lib.krk_sha256_resume_dev_on_host(h.ctypes.data_as(C.POINTER(C.c_uint32)), prev,
                                                        C.c_void_p(buf.ptr + prev), c - prev, int(c == L),
                                                        out.ctypes.data_as(C.POINTER(C.c_uint8)), None))
            prev = c
        assert bytes(out) == hashlib.sha256(data.tobytes()).digest(), L
        buf.free()
