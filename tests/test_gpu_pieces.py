"""GPU parity: piece CRC-32 (core.calcPieceSums, core/metainfo.go:157-179) through
the C ABI vs the CPU oracle, bit-exact.  Mirrors the reference's piece-length
edge cases (core/metainfo_test.go:25-46: 10/3, 8/2, ...) and adds lane/step/item
boundaries of the HIP kernel (64 B segments, 4 KiB wave steps, 256 KiB items)."""
import ctypes as C
import os

import numpy as np
import pytest

from kraken_amd import core
from kraken_amd import device as D

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 2, 3, 4, 7, 8, 10, 15, 16, 17, 63, 64, 65, 127, 255, 256, 4031, 4032, 4095, 4096, 4097,
        8191, 8192, 12345, 65536 + 7, 262143, 262144, 262145, 524288 + 4096 + 3, 1 << 20, (1 << 20) + 13]
PIECES = [1, 2, 3, 8, 10, 16, 4096, 4100, 65536, 262144, 1 << 20, 4 << 20]


def _check_arena(arena, orc, variant=0):
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)
    D.synchronize()
    sums = out.sums.to_host(np.uint32, arena.total_pieces)
    for i, L in enumerate(arena.lengths):
        L, P = int(L), int(arena.piece_lengths[i])
        ref = orc.calc_piece_sums(orc.synth(int(arena.blob_ids[i]), L, variant=variant), P)[1]
        o, n = int(arena.sums_off[i]), int(arena.n_pieces[i])
        assert n == len(ref), (L, P)
        got = sums[o:o + n]
        bad = np.nonzero(got != ref)[0]
        assert bad.size == 0, f"L={L} P={P}: {bad.size} bad pieces, first {bad[:5]}"


@pytest.mark.parametrize("P", PIECES)
def test_piece_sums_edge_lengths(gpu, orc, P):
    lens = [L for L in EDGE if L // P <= 4096]
    arena = D.BlobArena(lens, P, blob_ids=range(100, 100 + len(lens)))
    _check_arena(arena, orc)


@pytest.mark.parametrize("misalign", [1, 3, 8])
def test_piece_sums_unaligned(gpu, orc, misalign):
    lens = [5, 100, 4096 + 5, 70000, 300000]
    arena = D.BlobArena(lens, 65536, blob_ids=range(7, 7 + len(lens)), misalign=misalign)
    _check_arena(arena, orc)


def test_piece_sums_alnum_mixed_piece_lengths(gpu, orc):
    # randutil.Text-like content (core/fixtures.go:46-61) and one piece length per blob
    lens = [256, 10, 8, 1000, 99999, 1 << 20, 3 << 20]
    pls = [8, 3, 2, 7, 4096, 1 << 20, 1 << 20]
    arena = D.BlobArena(lens, pls, blob_ids=range(50, 57), variant=1)
    _check_arena(arena, orc, variant=1)


def test_piece_sums_many_small_blobs(gpu, orc):
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 300000, size=300).tolist()
    arena = D.BlobArena(lens, 262144, blob_ids=range(1000, 1300))
    _check_arena(arena, orc)


def test_piece_sums_c1_one_gib(gpu, orc):
    """BASELINE config C1 (1 GiB blob, 4 MiB pieces = 256 sums) at full size."""
    L, P = 1 << 30, 4 << 20
    arena = D.BlobArena([L], P, blob_ids=[0])
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)
    D.synchronize()
    got = out.sums.to_host(np.uint32, 256)
    data = orc.synth(0, L)
    ref = np.array([orc.crc32_clmul(data[i * P:(i + 1) * P]) for i in range(256)], dtype=np.uint32)
    assert np.array_equal(got, ref)


def test_piece_length_must_be_positive(gpu):
    arena = D.BlobArena([10], 3, blob_ids=[1])
    bad = arena.blob_structs()
    bad[0].piece_length = 0
    with pytest.raises(core.KrakenError, match="piece length must be positive"):
        from kraken_amd._capi import check, lib
        check(lib.krk_piece_sums_dev(bad, 1, 0, None))


def test_sums_offsets_are_respected(gpu, orc):
    # two blobs writing into an interleaved, gapped sums layout
    arena = D.BlobArena([5000, 9000], 1000, blob_ids=[3, 4])
    structs = arena.blob_structs()
    structs[0].sums_offset = 20
    structs[1].sums_offset = 2
    buf = D.DeviceBuffer(64 * 4)
    buf.from_host(np.full(64, 0xDEADBEEF, dtype=np.uint32))
    from kraken_amd._capi import check, lib
    check(lib.krk_piece_sums_dev(structs, 2, buf.ptr, None))
    D.synchronize()
    got = buf.to_host(np.uint32, 64)
    r0 = orc.calc_piece_sums(orc.synth(3, 5000), 1000)[1]
    r1 = orc.calc_piece_sums(orc.synth(4, 9000), 1000)[1]
    assert np.array_equal(got[20:25], r0)
    assert np.array_equal(got[2:11], r1)


def test_verify_pieces(gpu, orc):
    arena = D.BlobArena([300000], 65536, blob_ids=[9])
    ref = orc.calc_piece_sums(orc.synth(9, 300000), 65536)[1].copy()
    ref[2] ^= 1
    ok = np.zeros(len(ref), dtype=np.uint8)
    from kraken_amd._capi import check, lib
    b = arena.blob_structs()
    check(lib.krk_verify_pieces_dev(b, ref.ctypes.data_as(C.POINTER(C.c_uint32)),
                                    ok.ctypes.data_as(C.POINTER(C.c_uint8)), None))
    assert ok.tolist() == [1, 1, 0, 1, 1]


def test_piece_hash_update_matches_crc32(gpu, orc):
    h = core.PieceHash()
    parts = [os.urandom(n) for n in (0, 1, 17, 4096, 100000, 3)]
    for p in parts:
        h.Write(p)
    assert h.Sum32() == orc.crc32(b"".join(parts))
    h.Write(b"more")
    assert h.Sum32() == orc.crc32(b"".join(parts) + b"more")


def test_piece_sums_host_batch(gpu, orc):
    """End-to-end host path (pinned staging, windows smaller than the data)."""
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (0, 1, 777, 5 << 20, 3 << 20 + 11)]
    pls = [4, 4, 100, 1 << 20, 4 << 20]
    from kraken_amd._capi import check, krk_blob, lib
    offs, o = [], 0
    for d, p in zip(datas, pls):
        offs.append(o)
        o += int(lib.krk_num_pieces(d.size, p))
    arr = (krk_blob * len(datas))()
    for i, (d, p) in enumerate(zip(datas, pls)):
        arr[i] = krk_blob(d.ctypes.data if d.size else None, d.size, p, offs[i])
    sums = np.zeros(o, dtype=np.uint32)
    os.environ["KRK_WINDOW_MB"] = "2"
    try:
        check(lib.krk_piece_sums_host(arr, len(datas), sums.ctypes.data_as(C.POINTER(C.c_uint32))))
    finally:
        del os.environ["KRK_WINDOW_MB"]
    for i, (d, p) in enumerate(zip(datas, pls)):
        ref = orc.calc_piece_sums(d, p)[1]
        assert np.array_equal(sums[offs[i]:offs[i] + len(ref)], ref), i
