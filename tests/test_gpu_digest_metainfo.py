"""GPU parity: SHA-256 digests (core.Digester, core/digester.go:28-72) and
NewMetaInfo / InfoHash (core/metainfo.go:53-79) through the C ABI vs hashlib and
the CPU oracle, bit-exact.  KATs from core/digester_test.go:27-28 and
core/metainfo_test.go:61-76."""
import ctypes as C
import hashlib
import io
import os

import numpy as np
import pytest

from kraken_amd import core
from kraken_amd import device as D
from kraken_amd._capi import check, lib

pytestmark = pytest.mark.gpu

SHA_LENS = list(range(0, 130)) + [183, 184, 191, 192, 255, 256, 1000, 4096, 65535, 65536, 1 << 20, (1 << 20) + 55]


def test_digester_kat(gpu):
    d = core.NewDigester()
    assert d.FromBytes(b"test").Hex() == "9f86d081884c7d659a2feaa0c55ad015a3bf4f1b2b0b822cd15d6c15b0f00a08"
    assert core.NewDigester().Digest().String() == core.DigestEmptyTar


def test_digester_reader_and_tee(gpu):
    data = os.urandom(300000)
    assert core.NewDigester().FromReader(io.BytesIO(data)).Hex() == hashlib.sha256(data).hexdigest()
    d = core.NewDigester()
    r = d.Tee(io.BytesIO(data))
    w = io.BytesIO()
    while True:
        b = r.read(32768)
        if not b:
            break
        w.write(b)
    assert w.getvalue() == data
    assert d.Digest().Hex() == hashlib.sha256(data).hexdigest()


def test_digester_no_reset(gpu):
    """Digest() does not reset; FromBytes twice hashes the concatenation."""
    d = core.NewDigester()
    a, b = os.urandom(100), os.urandom(70000)
    assert d.FromBytes(a).Hex() == hashlib.sha256(a).hexdigest()
    assert d.FromBytes(b).Hex() == hashlib.sha256(a + b).hexdigest()
    assert d.Digest().Hex() == hashlib.sha256(a + b).hexdigest()


def test_digester_large_chunked(gpu):
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, size=40 << 20, dtype=np.uint8).tobytes()
    d = core.NewDigester()
    pos = 0
    for n in rng.integers(1, 3 << 20, size=100):
        d._write(data[pos:pos + int(n)])
        pos += int(n)
        if pos >= len(data):
            break
    d._write(data[pos:])
    assert d.Digest().Hex() == hashlib.sha256(data).hexdigest()


def test_sha256_dev_batch_lengths(gpu, orc):
    arena = D.BlobArena(SHA_LENS, 4096, blob_ids=range(len(SHA_LENS)))
    out = D.BatchOutputs(arena)
    D.sha256(arena, out)
    D.synchronize()
    got = out.digests.to_host(np.uint8, 32 * len(SHA_LENS)).reshape(-1, 32)
    for i, L in enumerate(SHA_LENS):
        ref = hashlib.sha256(orc.synth(i, L).tobytes()).digest()
        assert bytes(got[i]) == ref, L


@pytest.mark.parametrize("misalign", [1, 4, 8])
def test_sha256_dev_unaligned(gpu, orc, misalign):
    lens = [0, 55, 56, 64, 65, 1000, 100003]
    arena = D.BlobArena(lens, 4096, blob_ids=range(20, 27), misalign=misalign)
    out = D.BatchOutputs(arena)
    if os.environ.get("KRK_TEST_VERBOSE"):
        print(f"arena=0x{arena.buf.ptr:x}+{arena.nbytes} digests=0x{out.digests.ptr:x} "
              f"offsets={arena.offsets.tolist()}", flush=True)
    D.sha256(arena, out)
    D.synchronize()
    got = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
    for i, L in enumerate(lens):
        assert bytes(got[i]) == hashlib.sha256(orc.synth(20 + i, L).tobytes()).digest(), L


def test_sha256_host_batch_windowed(gpu):
    rng = np.random.default_rng(11)
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (0, 1, 64, 1000, 3 << 20, 5 << 20 + 3)]
    ptrs = (C.c_void_p * len(datas))(*[d.ctypes.data if d.size else None for d in datas])
    lens = np.array([d.size for d in datas], dtype=np.uint64)
    out = np.zeros((len(datas), 32), dtype=np.uint8)
    os.environ["KRK_WINDOW_MB"] = "1"
    try:
        check(lib.krk_sha256_host(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), len(datas),
                                  out.ctypes.data_as(C.POINTER(C.c_uint8))))
    finally:
        del os.environ["KRK_WINDOW_MB"]
    for i, d in enumerate(datas):
        assert bytes(out[i]) == hashlib.sha256(d.tobytes()).digest(), i


def test_metainfo_digest_batch(gpu, orc):
    """Both products in one call (the two passes of uploader.verify + Generate)."""
    lens = [0, 1, 1000, 4 << 20, (4 << 20) + 1, 9_999_999]
    arena = D.BlobArena(lens, 4 << 20, blob_ids=range(200, 206))
    out = D.BatchOutputs(arena)
    D.metainfo_digest(arena, out)
    D.synchronize()
    sums = out.sums.to_host(np.uint32, arena.total_pieces)
    dg = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
    for i, L in enumerate(lens):
        data = orc.synth(200 + i, L)
        assert bytes(dg[i]) == orc.sha256(data)
        ref = orc.calc_piece_sums(data, 4 << 20)[1]
        o = int(arena.sums_off[i])
        assert np.array_equal(sums[o:o + len(ref)], ref)


@pytest.mark.parametrize("size,pl", [(10, 3), (8, 2), (256, 8), (236, 4194304), (0, 4), (1 << 20, 4096),
                                     ((64 << 20) + 5, 4 << 20), (100_000, 100_000)])
def test_new_metainfo_matches_oracle(gpu, orc, size, pl):
    """NewMetaInfo over a reader (core/fixtures.go SizedBlobFixture shape)."""
    data = orc.synth(size, size, variant=1).tobytes()
    d = core.NewSHA256DigestFromHex(hashlib.sha256(data).hexdigest())
    mi = core.NewMetaInfo(d, io.BytesIO(data), pl)
    length, ref = orc.calc_piece_sums(data, pl)
    assert mi.Length() == length == size
    assert np.array_equal(mi.PieceSums(), ref)
    assert bytes(mi.InfoHash()) == orc.info_hash(pl, ref, d.Hex(), size)
    for i in range(-1, mi.NumPieces() + 1):
        assert mi.GetPieceLength(i) == orc.get_piece_length(size, pl, len(ref), i)


def test_metainfo_get_piece_length_table(gpu):
    """core/metainfo_test.go:25-46."""
    cases = [(10, 3, 0, 3), (10, 3, 3, 1), (8, 2, 3, 2), (10, 3, 1, 3), (10, 3, 4, 0), (10, 3, -1, 0)]
    for size, pl, i, want in cases:
        data = os.urandom(size)
        mi = core.NewMetaInfo(core.NewDigester().FromBytes(data), data, pl)
        assert mi.GetPieceLength(i) == want


def test_metainfo_serialization_roundtrip(gpu):
    data = os.urandom(256)
    d = core.NewDigester().FromBytes(data)
    mi = core.NewMetaInfo(d, data, 8)
    back = core.DeserializeMetaInfo(mi.Serialize())
    assert back.Digest() == d and back.InfoHash() == mi.InfoHash()


def test_new_metainfo_bad_piece_length(gpu):
    with pytest.raises(ValueError, match="piece length must be positive"):
        core.NewMetaInfo(core.NewDigester().FromBytes(b"x"), b"x", 0)


def test_generator_generate_and_batch(gpu, orc, tmp_path):
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    blobs = [os.urandom(n) for n in (0, 17, 3 << 20, (5 << 20) + 1)]
    ds = [cas.WriteCacheFile(b) for b in blobs]
    g = metainfogen.New({0: 1 << 20, 4 << 20: 4 << 20}, cas)
    for d, b in zip(ds, blobs):
        g.Generate(d)
        mi = core.DeserializeMetaInfo(open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read())
        pl = 1 << 20 if len(b) < 4 << 20 else 4 << 20
        ref = orc.calc_piece_sums(b, pl)[1]
        assert bytes(mi.InfoHash()) == orc.info_hash(pl, ref, d.Hex(), len(b))
    mis = g.GenerateBatch(ds)
    for mi, d, b in zip(mis, ds, blobs):
        pl = mi.PieceLength()
        assert bytes(mi.InfoHash()) == orc.info_hash(pl, orc.calc_piece_sums(b, pl)[1], d.Hex(), len(b))


@pytest.mark.parametrize("window_mb", [1, 256])
def test_metainfo_digest_host_end_to_end(gpu, orc, window_mb):
    """krk_metainfo_digest_host: host buffers, one PCIe pass feeding both kernels,
    several windows per blob at 1 MiB (midstate chaining + CRC across windows)."""
    rng = np.random.default_rng(window_mb)
    lens = [0, 1, 63, 64, 65, 4095, 1 << 20, (3 << 20) + 17, 5_000_001]
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in lens]
    pls = [4096, 3, 64, 64, 10, 4096, 1 << 18, 1 << 20, 4 << 20]
    os.environ["KRK_WINDOW_MB"] = str(window_mb)
    try:
        sums, dg = D.metainfo_digest_host(datas, pls)
    finally:
        del os.environ["KRK_WINDOW_MB"]
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), lens[i]
        ref = orc.calc_piece_sums(d, pls[i])[1]
        assert np.array_equal(sums[i], ref), lens[i]


def test_metainfo_digest_chunks_dev(gpu, orc):
    """krk_metainfo_digest_chunks_dev: blobs advanced by uneven 64-multiple chunks
    over several calls (blobs finishing at different calls) == one-shot results."""
    rng = np.random.default_rng(5)
    lens = [0, 1, 64, 200, 4096, 70_000, 1 << 20, (1 << 20) + 3]
    pls = [8, 3, 64, 7, 1000, 4096, 1 << 18, 100_000]
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in lens]
    buf = D.DeviceBuffer(sum(lens) + 16 * len(lens))
    base, off = [], 0
    for d in datas:
        base.append(off)
        buf.from_host(d, off)
        off += (d.size + 15) // 16 * 16
    cb = D.ChunkedBatch(lens, pls)
    pos = [0] * len(lens)
    started = [False] * len(lens)
    while not all(started[i] and pos[i] >= lens[i] for i in range(len(lens))):
        items = []
        for i, L in enumerate(lens):
            if started[i] and pos[i] >= L:
                continue
            step = int(rng.integers(1, 5000)) * 64
            take = min(step, L - pos[i])
            items.append((i, buf.ptr + base[i] + pos[i], pos[i], take))
            pos[i] += take
            started[i] = True
        cb.step(items)
    D.synchronize()
    dg = cb.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
    sums = cb.sums.to_host(np.uint32, max(cb.total_pieces, 1))
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), lens[i]
        ref = orc.calc_piece_sums(d, pls[i])[1]
        o = int(cb.sums_off[i])
        assert np.array_equal(sums[o:o + len(ref)], ref), lens[i]


def test_synth_fill_chunks_matches_spec(gpu, orc):
    """Batched window generator == the synthetic-blob spec (oracle/oracle.c orc_synth_fill)."""
    specs = [(3, 0, 100), (3, 100, 1 << 16), (9, 64, 4097), (11, 7, 33), (12, 1 << 20, 1_000_003)]
    buf = D.DeviceBuffer(sum(n + 16 for _, _, n in specs))
    items, off = [], 0
    for b, o, n in specs:
        items.append((b, buf.ptr + off, o, n))
        off += (n + 15) // 16 * 16
    D.synth_fill_chunks(items)
    D.synchronize()
    for (b, o, n), (_, ptr, _, _) in zip(specs, items):
        got = buf.to_host(np.uint8, n, ptr - buf.ptr)
        assert np.array_equal(got, orc.synth(b, n, offset=o)), (b, o, n)


def test_verify_and_generate_batch(gpu, orc, tmp_path):
    """Fused upload verify + Generate (one PCIe pass): a corrupted upload is rejected
    with the reference's message, the others are committed with byte-identical
    _torrentmeta to the two-pass path."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    g = metainfogen.New({0: 1 << 20, 4 << 20: 4 << 20}, cas)
    blobs = [os.urandom(n) for n in (0, 5, 1 << 20, (4 << 20) + 7, 3_000_001)]
    want = [core.NewSHA256DigestFromHex(hashlib.sha256(b).hexdigest()) for b in blobs]
    bad = bytearray(blobs[3])
    bad[12345] ^= 1
    ups = list(zip(want, blobs)) + [(want[3], bytes(bad))]
    res = g.VerifyAndGenerateBatch(ups)
    assert isinstance(res[-1], ValueError) and "doesn't match parameter" in str(res[-1])
    for mi, d, b in zip(res[:-1], want, blobs):
        pl = 1 << 20 if len(b) < 4 << 20 else 4 << 20
        assert bytes(mi.InfoHash()) == orc.info_hash(pl, orc.calc_piece_sums(b, pl)[1], d.Hex(), len(b))
        two_pass = core.NewMetaInfo(d, b, pl)
        assert open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read() == two_pass.Serialize()
        assert open(os.path.join(cas._dir(d.Hex()), "data"), "rb").read() == b


def test_verify_and_generate_uploads_from_files(gpu, orc, tmp_path):
    """The files form (krk_metainfo_digest_files: one read of each upload file feeds the
    digest and the piece sums): a corrupted upload is rejected with uploader.verify's
    message and stays in the upload dir, the others are moved into the CAS with
    _torrentmeta byte-identical to the two-pass path; an unreadable upload fails the batch
    with the reference's prefixes."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path / "cas"))
    up = tmp_path / "upload"
    up.mkdir()
    g = metainfogen.New({0: 1 << 20, 4 << 20: 4 << 20}, cas)
    blobs = [os.urandom(n) for n in (0, 5, 1 << 20, (4 << 20) + 7, 3_000_001)]
    want = [core.NewSHA256DigestFromHex(hashlib.sha256(b).hexdigest()) for b in blobs]
    bad = bytearray(blobs[3])
    bad[777] ^= 4
    ups = []
    for i, b in enumerate(blobs + [bytes(bad)]):
        p = up / f"u{i}"
        p.write_bytes(b)
        ups.append((want[i] if i < len(blobs) else want[3], str(p)))
    res = g.VerifyAndGenerateUploads(ups)
    assert isinstance(res[-1], ValueError) and "doesn't match parameter" in str(res[-1])
    assert os.path.exists(ups[-1][1])  # the rejected upload is not committed
    for mi, d, b, (_, p) in zip(res[:-1], want, blobs, ups):
        pl = 1 << 20 if len(b) < 4 << 20 else 4 << 20
        assert bytes(mi.InfoHash()) == orc.info_hash(pl, orc.calc_piece_sums(b, pl)[1], d.Hex(), len(b))
        assert open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read() == core.NewMetaInfo(d, b, pl).Serialize()
        assert open(os.path.join(cas._dir(d.Hex()), "data"), "rb").read() == b and not os.path.exists(p)
    with pytest.raises(IOError, match="get upload file: "):
        g.VerifyAndGenerateUploads([(want[1], str(up / "missing"))])


def test_verify_and_generate_uploads_conflicts(gpu, orc, tmp_path):
    """a verified upload whose blob is already cached, or a second upload of one
    digest in the same batch, is that upload's 409 (uploader.commit, origin/blobserver/
    uploader.go:96-104) with its upload file deleted (ca_store.go:79-86); the batch goes on
    and every other upload gets its _torrentmeta."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path / "cas"))
    up = tmp_path / "upload"
    up.mkdir()
    g = metainfogen.New({0: 1 << 20}, cas)
    blobs = [os.urandom(n) for n in (3_000_001, 12345, 1 << 20)]
    want = [core.NewSHA256DigestFromHex(hashlib.sha256(b).hexdigest()) for b in blobs]
    cached = cas.WriteCacheFile(blobs[1])  # blob 1 is in the CAS already
    assert cached == want[1]
    order = [0, 1, 2, 0]  # blob 0 twice in the batch
    ups = []
    for k, i in enumerate(order):
        p = up / f"u{k}"
        p.write_bytes(blobs[i])
        ups.append((want[i], str(p)))
    res = g.VerifyAndGenerateUploads(ups)
    assert isinstance(res[1], FileExistsError) and isinstance(res[3], FileExistsError), res
    for k in (0, 2):
        i = order[k]
        b, d = blobs[i], want[i]
        assert bytes(res[k].InfoHash()) == orc.info_hash(1 << 20, orc.calc_piece_sums(b, 1 << 20)[1], d.Hex(), len(b))
        assert open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read() == \
            core.NewMetaInfo(d, b, 1 << 20).Serialize()
        assert open(os.path.join(cas._dir(d.Hex()), "data"), "rb").read() == b
    assert not any(os.path.exists(p) for _, p in ups)  # committed or conflicting: every upload file is gone
    assert open(os.path.join(cas._dir(want[1].Hex()), "data"), "rb").read() == blobs[1]


def _go_json(pl, sums, name, length):
    """encoding/json of metaInfoJSON{info} (core/metainfo.go:125-134), written out
    independently of core.MetaInfo.Serialize: declared field order, compact, nil
    slice -> null."""
    ps = "null" if sums is None else "[" + ",".join(str(int(x)) for x in sums) + "]"
    return ('{"Info":{"PieceLength":%d,"PieceSums":%s,"Name":"%s","Length":%d}}' % (pl, ps, name, length)).encode()


def test_regenerate_all_cas_sidecars(gpu, orc, tmp_path):
    """Whole-CAS _torrentmeta regeneration in the reference's
    shard layout, byte-identical sidecars, only changed ones rewritten."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    rng = np.random.default_rng(21)
    lens = [0, 1, 4095, 65536, 1 << 20, (1 << 20) + 3, (3 << 20) + 7, 9 << 20]
    blobs = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    ds = [cas.WriteCacheFile(b) for b in blobs]
    for d in ds:  # <hex[0:2]>/<hex[2:4]>/<hex>/data (lib/store/base/file_entry.go:176-189)
        h = d.Hex()
        assert os.path.exists(tmp_path / h[:2] / h[2:4] / h / "data")
    assert cas.ListNames() == sorted(d.Hex() for d in ds)
    cfg = {0: 1 << 20, 8 << 20: 4 << 20}
    g = metainfogen.New(cfg, cas)
    assert g.RegenerateAll(batch_bytes=4 << 20) == {"blobs": len(ds), "changed": len(ds)}
    for d, b in zip(ds, blobs):
        pl = 1 << 20 if len(b) < 8 << 20 else 4 << 20
        ref = orc.calc_piece_sums(b, pl)[1] if len(b) else None
        got = open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read()
        assert got == _go_json(pl, ref, d.Hex(), len(b))
    assert g.RegenerateAll() == {"blobs": len(ds), "changed": 0}
    # CLI over the same directory with another piece-length table rewrites everything
    assert metainfogen.main([str(tmp_path), "--piece-lengths", "0:65536"]) == 0
    for d, b in zip(ds, blobs):
        ref = orc.calc_piece_sums(b, 65536)[1] if len(b) else None
        got = open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read()
        assert got == _go_json(65536, ref, d.Hex(), len(b))


@pytest.fixture
def sha_plan():
    """Sets a process-wide SHA-256 launch plan (krk_set_sha_plan), restores AUTO after."""
    from kraken_amd._capi import lib as L

    def set_plan(p):
        check(L.krk_set_sha_plan(p))
    yield set_plan
    check(L.krk_set_sha_plan(0))


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6])
def test_sha_launch_plans_bit_exact(gpu, orc, variant, sha_plan):
    """Every production SHA-256 plan (KRK_SHA_PLAN_*: one / two / eight lanes per
    stream; one / two producer-consumer pairs per workgroup) on a batch of mixed lengths and
    alignments, one-shot and from midstates (chunked), against hashlib."""
    sha_plan(variant)
    rng = np.random.default_rng(int(variant))
    lens = [int(x) for x in rng.integers(0, 300_000, 300)] + [0, 1, 55, 56, 63, 64, 65, 119, 120, 128]
    arena = D.BlobArena(lens, 1 << 16, blob_ids=range(900, 900 + len(lens)), misalign=int(variant) % 3)
    out = D.BatchOutputs(arena)
    D.sha256(arena, out)
    D.synchronize()
    dg = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
    for i, L in enumerate(lens):
        assert bytes(dg[i]) == hashlib.sha256(orc.synth(900 + i, L).tobytes()).digest(), (variant, i, L)
    # chunked: midstates carried in HBM across three calls
    cb = D.ChunkedBatch(lens, 1 << 16)
    pos = [0] * len(lens)
    for step in range(3):
        items = []
        for i, L in enumerate(lens):
            if pos[i] == L and (L or step):
                continue  # finished in an earlier call
            take = L - pos[i] if step == 2 else min(L - pos[i], 64 * int(rng.integers(0, 1500)))
            items.append((i, arena.buf.ptr + int(arena.offsets[i]) + pos[i], pos[i], take))
            pos[i] += take
        cb.step(items)
    D.synchronize()
    cdg = cb.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
    assert np.array_equal(cdg, dg), variant


class _ReaderOnlyCAS:
    """A CAS without GetCacheFilePath: GenerateBatch takes the reader route."""

    def __init__(self, cas, stat_extra=0):
        self.cas, self.stat_extra = cas, stat_extra

    def GetCacheFileStat(self, h):
        return self.cas.GetCacheFileStat(h)

    def GetCacheFileReader(self, h):
        return self.cas.GetCacheFileReader(h)

    def SetCacheFileMetadata(self, h, mi):
        return self.cas.SetCacheFileMetadata(h, mi)


@pytest.mark.parametrize("direct,window_mb", [("0", 1), ("1", 1), ("0", 512), ("1", 512)])
def test_generate_batch_from_files(gpu, orc, tmp_path, direct, window_mb):
    """krk_piece_sums_files (cache files read straight into pinned staging, pread
    threads or O_DIRECT) == the reader route == the oracle, with files split over
    1 MiB windows and sizes off every alignment."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    rng = np.random.default_rng(int(direct) * 7 + window_mb)
    lens = [0, 1, 15, 4095, 4096, 4097, 65537, (1 << 20) - 1, 1 << 20, (1 << 20) + 4097, (3 << 20) + 5, 9_000_001]
    blobs = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    ds = [cas.WriteCacheFile(b) for b in blobs]
    cfg = {0: 65536, 1 << 20: 1 << 20, 8 << 20: 4 << 20}
    os.environ["KRK_WINDOW_MB"], os.environ["KRK_FILE_DIRECT"] = str(window_mb), direct
    try:
        mis = metainfogen.New(cfg, cas).GenerateBatch(ds)
        mis_r = metainfogen.New(cfg, _ReaderOnlyCAS(cas)).GenerateBatch(ds)
    finally:
        del os.environ["KRK_WINDOW_MB"], os.environ["KRK_FILE_DIRECT"]
    for mi, mr, d, b in zip(mis, mis_r, ds, blobs):
        pl = mi.PieceLength()
        ref = orc.calc_piece_sums(b, pl)[1]
        assert mi.InfoHash() == mr.InfoHash()
        assert bytes(mi.InfoHash()) == orc.info_hash(pl, ref, d.Hex(), len(b)), len(b)
        assert mi.Serialize() == open(os.path.join(cas._dir(d.Hex()), "_torrentmeta"), "rb").read()


def test_generate_batch_file_errors(gpu, tmp_path):
    """Generate's error prefixes (generator.go:41-58) on the file route: a missing
    cache file -> "cache stat: ...", a file shorter than its stat size ->
    "create metainfo: read blob: <path>: unexpected EOF"."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    d = cas.WriteCacheFile(os.urandom(100_000))
    g = metainfogen.New({0: 4096}, cas)
    with pytest.raises(IOError, match="^cache stat: "):
        g.GenerateBatch([core.NewSHA256DigestFromHex("ab" * 32)])

    class Lying(metainfogen.DirCAS):
        def GetCacheFileStat(self, h):
            st = super().GetCacheFileStat(h)
            return os.stat_result((st.st_mode, st.st_ino, st.st_dev, st.st_nlink, st.st_uid, st.st_gid,
                                   st.st_size + 5000, st.st_atime, st.st_mtime, st.st_ctime))

    with pytest.raises(IOError, match="^create metainfo: read blob: .*: unexpected EOF"):
        metainfogen.New({0: 4096}, Lying(str(tmp_path))).GenerateBatch([d])


@pytest.mark.parametrize("misalign", [0, 3])
def test_sha_host_offload_bit_exact(gpu, orc, misalign):
    """krk_set_sha_host_offload: the longest blobs are hashed on host threads (read out of
    HBM in 8 MiB double-buffered chunks: lengths on, around and past chunk edges), the
    rest on the GPU; digests (krk_sha256_dev, krk_metainfo_digest_dev) and piece sums
    equal hashlib / the oracle."""
    big = [(40 << 20) + 13, 17 << 20, 8 << 20, (8 << 20) + 64, (16 << 20) - 1]
    lens = big + [65536 + 7 * i for i in range(200)] + [0, 1, 63, 64]
    ids = list(range(5000, 5000 + len(lens)))
    P = 1 << 20
    host_idx = D.sha_offload_plan(lens, 8, 256)[0]
    assert set(host_idx.tolist()) >= set(range(len(big)))  # the long ones go to the host
    arena = D.BlobArena(lens, P, blob_ids=ids, misalign=misalign)
    out = D.BatchOutputs(arena)
    want = [hashlib.sha256(orc.synth(b, L).tobytes()).digest() for b, L in zip(ids, lens)]
    try:
        D.set_sha_host_offload(8)
        for fn in (D.sha256, D.metainfo_digest):
            out.digests.from_host(np.zeros(32 * len(lens), dtype=np.uint8))
            fn(arena, out)
            D.synchronize()
            dg = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
            for i in range(len(lens)):
                assert bytes(dg[i]) == want[i], (fn.__name__, i, lens[i])
        sums = out.sums.to_host(np.uint32, max(arena.total_pieces, 1))
        for i, (b, L) in enumerate(zip(ids, lens)):
            ref = orc.calc_piece_sums(orc.synth(b, L), P)[1]
            o = int(arena.sums_off[i])
            assert np.array_equal(sums[o:o + len(ref)], ref), i
    finally:
        D.set_sha_host_offload(0)


@pytest.mark.parametrize("misalign", [0, 3])
def test_sha_tail_handoff_bit_exact(gpu, orc, misalign):
    """Tail handoff of the host offload: the GPU runs the first start[k] bytes of a chain and
    writes its midstate to page-locked host memory, a host thread reads it there and finishes
    the chain from HBM (prefix lengths are 64-byte multiples; tails end on, around and past
    the 8 MiB copy-chunk edges).  Rates set so the plan hands tails over whatever the box;
    digests (krk_sha256_dev, krk_metainfo_digest_dev) equal hashlib, piece sums the oracle."""
    lens = [(24 << 20) + 13 * k for k in range(40)] + [(8 << 20) + 64, 4096 + 1, 0, 1, 63, 64]
    ids = list(range(7000, 7000 + len(lens)))
    P = 1 << 20
    R = D.planner_rates()
    rates = dict(R, sha_stream_bps=[50e6, 50e6, 35e6], host_sha_bps=0.2e9, d2h_bps=50e9, h2d_bps=50e9, cus=256)
    arena = D.BlobArena(lens, P, blob_ids=ids, misalign=misalign)
    out = D.BatchOutputs(arena)
    want = [hashlib.sha256(orc.synth(b, L).tobytes()).digest() for b, L in zip(ids, lens)]
    try:
        D.set_planner_rates(rates)
        idx, start, end_s, gpu_s = D.sha_tail_plan(lens, 8)
        assert idx.size and (start > 0).any() and end_s < 0.95 * gpu_s
        D.set_sha_host_offload(8)
        for fn in (D.sha256, D.metainfo_digest):
            out.digests.from_host(np.zeros(32 * len(lens), dtype=np.uint8))
            fn(arena, out)
            D.synchronize()
            tail = D.sha_last_tail()
            assert tail["chains"] > 0 and tail["gpu_prefix_bytes"] > 0, (fn.__name__, tail)
            dg = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
            for i in range(len(lens)):
                assert bytes(dg[i]) == want[i], (fn.__name__, i, lens[i])
        sums = out.sums.to_host(np.uint32, max(arena.total_pieces, 1))
        for i, (b, L) in enumerate(zip(ids, lens)):
            ref = orc.calc_piece_sums(orc.synth(b, L), P)[1]
            o = int(arena.sums_off[i])
            assert np.array_equal(sums[o:o + len(ref)], ref), i
    finally:
        D.set_sha_host_offload(0)
        D.set_planner_rates(None)


@pytest.mark.parametrize("window_mb", ["1", None])
def test_sha_host_offload_host_buffers(gpu, orc, window_mb):
    """The host-buffer entry points with the offload on: the longest blobs are worked on
    in place on host threads and never uploaded (krk_sha256_host hashes them,
    krk_metainfo_digest_host hashes them and computes their piece sums on the host, the
    rest -- including the empty blob -- go through the windows); digests and sums equal
    hashlib / oracle."""
    rng = np.random.default_rng(31)
    sizes = [(24 << 20) + 5, 9 << 20, 0, 1, 63, 64, 1000] + [70_000 + 13 * i for i in range(60)]
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in sizes]
    for mode in (D.OFFLOAD_HOST_SHA, D.OFFLOAD_HOST_WHOLE):
        host = set(D.sha_offload_plan(sizes, 4, mode=mode)[0].tolist())
        assert host >= {0, 1} and 2 not in host and len(host) < len(sizes) - 1
    ptrs = (C.c_void_p * len(datas))(*[d.ctypes.data if d.size else None for d in datas])
    lens = np.array(sizes, dtype=np.uint64)
    want = [hashlib.sha256(d.tobytes()).digest() for d in datas]
    if window_mb:
        os.environ["KRK_WINDOW_MB"] = window_mb
    try:
        D.set_sha_host_offload(4)
        out = np.zeros((len(datas), 32), dtype=np.uint8)
        check(lib.krk_sha256_host(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), len(datas),
                                  out.ctypes.data_as(C.POINTER(C.c_uint8))))
        for i in range(len(datas)):
            assert bytes(out[i]) == want[i], ("sha256_host", i, sizes[i])
        sums, dg = D.metainfo_digest_host(datas, 1 << 20)
        for i, d in enumerate(datas):
            assert bytes(dg[i]) == want[i], ("metainfo_digest_host", i, sizes[i])
            assert np.array_equal(sums[i], orc.calc_piece_sums(d, 1 << 20)[1]), i
    finally:
        D.set_sha_host_offload(0)
        os.environ.pop("KRK_WINDOW_MB", None)


def test_host_whole_offload_piece_lengths(gpu, orc):
    """krk_metainfo_digest_host with the whole-blob host offload at several piece lengths
    (partial last pieces, 4 KiB and one-byte pieces): the MiB blobs are hashed and
    piece-summed on host threads, the small ones and the empty one go through the windows;
    piece sums and digests equal the oracle / hashlib."""
    rng = np.random.default_rng(5)
    sizes = [3 << 20, (2 << 20) + 1, 1 << 20, 4097, 0, 65, 1]
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in sizes]
    host = set(D.sha_offload_plan(sizes, 8, mode=D.OFFLOAD_HOST_WHOLE)[0].tolist())
    assert host >= {0, 1, 2} and 4 not in host
    try:
        D.set_sha_host_offload(8)
        for P in (1 << 20, 4096, 1):
            if P == 1:
                datas, sizes = datas[3:], sizes[3:]  # one-byte pieces: keep the piece count small
            sums, dg = D.metainfo_digest_host(datas, P)
            for i, d in enumerate(datas):
                assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), (P, i)
                assert np.array_equal(sums[i], orc.calc_piece_sums(d, P)[1]), (P, i)
    finally:
        D.set_sha_host_offload(0)
