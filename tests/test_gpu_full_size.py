"""GPU parity at BASELINE.json's full sizes, where the oracle cannot recompute
everything in seconds: sampled oracle checks plus size-independent properties.

* C2 (configs[1]: 1,000 x 100 MiB, 4 MiB pieces, 105 GB in HBM): ALL 1,000 digests and
  25,000 piece sums against the oracle's threaded runner (each blob regenerated on the
  host, ~7 s on 16 threads), and decomposition invariance over all blobs --
  the chunked path (SHA-256 from per-blob midstates, CRC items cut at chunk edges
  that split pieces) must give the same 1,000 digests and 25,000 sums as the
  one-shot path (two different work decompositions of the same bytes).
* C1 (configs[0]: one 1 GiB blob): the whole SHA-256 chain on one stream and the
  256 piece sums against hashlib / the oracle.
* C3 (configs[2]'s blob law, unscaled): 256 seeded blobs of 100 MiB - 1 GiB (151.7 GB,
  the bench's CPU-baseline sample, its longest 1.07 GB) through the production window
  machinery (kraken_amd.windowed.WindowedRun, 48 GiB windows), every digest and piece sum
  against the oracle; and rank 0's whole 8-GPU shard (2,500 blobs, 1.47 TB) through the
  GPU-only windows and the tail handoff, all digests and sums equal between the two.
* C4 (configs[3]: one 20 GiB blob, 256 KiB pieces): sampled pieces against the
  oracle (content regenerated at the piece's offset), and CRC linearity -- the
  81,920 piece sums combined with crc(A||B) = shift(crc(A), |B|) ^ crc(B) equal the
  GPU's CRC of the whole blob computed as ONE piece (81,920 work items XOR-reduced
  into a single sum).
"""
import hashlib
import zlib

import numpy as np
import pytest

from kraken_amd import device as D

pytestmark = pytest.mark.gpu

POLY = 0xEDB88320
ONE = 0x80000000  # the polynomial 1, bit-reflected (crc_math.hpp)


def _mulmod(a: int, b: int) -> int:
    p = 0
    for i in range(31, -1, -1):
        if (a >> i) & 1:
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


def _x8n(n: int) -> int:
    p, sq = ONE, ONE >> 8  # x^0, x^8
    while n:
        if n & 1:
            p = _mulmod(p, sq)
        sq = _mulmod(sq, sq)
        n >>= 1
    return p


def _combine(crcs, piece: int) -> int:
    """CRC of the concatenation of equal-length pieces from their CRCs
    (multiplication by the fixed x^(8*piece) through four byte tables)."""
    x = _x8n(piece)
    T = [[_mulmod(b << (8 * k), x) for b in range(256)] for k in range(4)]
    c = 0
    for s in crcs:
        c = T[0][c & 255] ^ T[1][(c >> 8) & 255] ^ T[2][(c >> 16) & 255] ^ T[3][c >> 24] ^ int(s)
    return c


def test_crc_combine_helper_matches_zlib():
    rng = np.random.default_rng(1)
    parts = [rng.integers(0, 256, 1000, dtype=np.uint8).tobytes() for _ in range(5)]
    assert _combine([zlib.crc32(p) for p in parts], 1000) == zlib.crc32(b"".join(parts))


def test_c2_full_size_decomposition_invariance(gpu, orc):
    n, L, P = 1000, 100 << 20, 4 << 20
    arena = D.BlobArena([L] * n, P)  # blob i = synthetic blob i, generated on the device
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    sums = out.sums.to_host(np.uint32, arena.total_pieces)
    dg = out.digests.to_host(np.uint8, 32 * n).reshape(n, 32)
    assert arena.total_pieces == 25_000
    for i in (0, 517, 999):
        data = orc.synth(i, L)
        assert bytes(dg[i]) == hashlib.sha256(data).digest(), i
        o = int(arena.sums_off[i])
        assert np.array_equal(sums[o:o + 25], orc.calc_piece_sums(data, P)[1]), i
    # every blob against the oracle: its threaded runner regenerates each
    # blob on the host and runs the reference's two passes, outputs kept
    _, dgo, (so, offo) = orc.baseline_run_lazy(list(range(n)), [L] * n, P, _threads(), passes=3)
    assert np.array_equal(dgo, dg)
    assert np.array_equal(so[:int(offo[-1])], sums)  # the arena's sums are laid out blob by blob
    cb = D.ChunkedBatch([L] * n, P)
    chunk = 3 * P + 64 * 1001  # a multiple of 64 that cuts pieces at varying offsets
    pos = 0
    while pos < L:
        take = min(chunk, L - pos)
        cb.step([(i, arena.buf.ptr + int(arena.offsets[i]) + pos, pos, take) for i in range(n)])
        pos += take
    D.synchronize()
    assert np.array_equal(cb.sums.to_host(np.uint32, arena.total_pieces), sums)
    assert np.array_equal(cb.digests.to_host(np.uint8, 32 * n).reshape(n, 32), dg)


def _threads():
    import os
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 32))


def test_c3_unscaled_sample_windows_match_oracle(gpu, orc):
    """C3 at unscaled lengths under a -m gpu test (it was only inside
    bench.py's cpu_baseline_c3): the bench's seeded 256-blob sample of the 20,000-blob law."""
    from kraken_amd.windowed import WindowedRun, c3_lengths
    lens_all = c3_lengths(20000)
    pick = np.sort(np.random.default_rng(0xC3).choice(20000, 256, replace=False))
    lens = [int(lens_all[i]) for i in pick]
    ids = [(2 << 40) + int(i) for i in pick]
    assert max(lens) >= 1_070_000_000 and sum(lens) > 150e9
    P = 4 << 20
    wr = WindowedRun(D, ids, lens, P, 48 << 30)
    try:
        wr.run()
        cb = wr.cb
        dg = cb.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
        sums = cb.sums.to_host(np.uint32, cb.total_pieces)
        offs = cb.sums_off.copy()
    finally:
        wr.close()
    _, dgo, (so, offo) = orc.baseline_run_lazy(ids, lens, P, _threads(), passes=3)
    assert np.array_equal(dgo, dg)
    for k in range(len(lens)):
        a, m = int(offs[k]), int(offo[k + 1] - offo[k])
        assert np.array_equal(sums[a:a + m], so[int(offo[k]):int(offo[k + 1])]), k


def test_c1_full_size_one_stream(gpu, orc):
    """C1 (configs[0]: one 1 GiB blob, 4 MiB pieces): NewMetaInfo + Digester of ONE
    stream at full size -- the SHA-256 chain runs 16,777,216 blocks on one eight-lane
    stream (~19 s), the CRC 256 pieces beside it."""
    L, P = 1 << 30, 4 << 20
    arena = D.BlobArena([L], P, blob_ids=[0])
    out = D.BatchOutputs(arena)
    assert D.sha_lanes_per_stream(1) == 8
    D.metainfo_digest(arena, out)
    D.synchronize()
    data = orc.synth(0, L)
    assert bytes(out.digests.to_host(np.uint8, 32)) == hashlib.sha256(data).digest()
    assert np.array_equal(out.sums.to_host(np.uint32, L // P), orc.calc_piece_sums(data, P)[1])


def test_c4_full_size_sampled_and_linear(gpu, orc):
    L, P = 20 << 30, 256 << 10
    arena = D.BlobArena([L], P, blob_ids=[0])
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)
    D.synchronize()
    n = L // P
    sums = out.sums.to_host(np.uint32, n)
    rng = np.random.default_rng(4)
    for pi in [0, 1, n // 2, n - 1] + rng.choice(n, 12, replace=False).tolist():
        assert int(sums[pi]) == orc.crc32_clmul(orc.synth(0, P, offset=pi * P)), pi
    # every one of the 81,920 pieces against the oracle: the arena's
    # bytes copied down 1 GiB at a time, each piece CRC'd by the oracle's PCLMUL restatement
    chunk = 1 << 30
    bad = []
    for c0 in range(0, L, chunk):
        h = arena.buf.to_host(np.uint8, chunk, offset=int(arena.offsets[0]) + c0)
        for k in range(chunk // P):
            if int(sums[c0 // P + k]) != orc.crc32_clmul(h[k * P:(k + 1) * P]):
                bad.append(c0 // P + k)
        del h
    assert not bad, bad[:10]
    # the same 20 GiB as ONE piece
    from kraken_amd._capi import check, krk_blob, lib
    one = (krk_blob * 1)(krk_blob(arena.buf.ptr + int(arena.offsets[0]), L, L, 0))
    s1 = D.DeviceBuffer(4)
    check(lib.krk_piece_sums_dev(one, 1, s1.ptr, None))
    D.synchronize()
    assert int(s1.to_host(np.uint32, 1)[0]) == _combine(sums, P)


def test_c3_shard_tail_handoff_whole_shard_equals_windows(gpu, orc):
    """C3's multi-GPU config at full size (C3 checked on 256 of 20,000
    blobs): rank 0's LPT shard of an 8-GPU run, 2,500 unscaled blobs (1.47 TB, longest
    1.07 GB), through the GPU-only windows and through the tail handoff (host threads
    finishing ~400 GB of chains on SHA-NI from the windows' midstates, the loop's copies and
    the GPU's CRCs of the stolen pieces).  Every one of the 2,500 digests and ~350,000 piece
    sums must agree between the two -- different work on different processors over the same
    bytes -- and the shard's shortest and longest blobs match the oracle."""
    from kraken_amd.shard import lpt_shard
    from kraken_amd.windowed import TAIL_CHUNK, TailHandoffRun, WindowedRun, c3_lengths
    lens_all = c3_lengths(20000)
    mine = lpt_shard(lens_all, 8)[0]
    ids = [(2 << 40) + int(i) for i in mine]
    lens = [int(lens_all[i]) for i in mine]
    P = 4 << 20
    assert len(lens) == 2500 and max(lens) > 1_070_000_000
    wr = WindowedRun(D, ids, lens, P, 10 << 30)
    try:
        wr.run()
        dg = wr.cb.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
        sums = wr.cb.sums.to_host(np.uint32, wr.cb.total_pieces)
        offs = wr.cb.sums_off.copy()
    finally:
        wr.close()
    tr = TailHandoffRun(D, ids, lens, P, min(10 << 30, len(lens) * TAIL_CHUNK), 15)
    try:
        tr.run()
        dg2 = tr.cb.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
        sums2 = tr.cb.sums.to_host(np.uint32, tr.cb.total_pieces)
        st = tr.stats
    finally:
        tr.close()
    assert st["host_bytes"] > 100e9 and st["resumed_from_midstate"] > 100, st
    assert np.array_equal(dg2, dg)
    assert np.array_equal(sums2, sums)
    for k in (int(np.argmin(lens)), int(np.argmax(lens))):
        data = orc.synth(ids[k], lens[k])
        assert bytes(dg[k]) == hashlib.sha256(data).digest(), k
        a = int(offs[k])
        want = orc.calc_piece_sums(data, P)[1]
        assert np.array_equal(sums[a:a + len(want)], want), k
