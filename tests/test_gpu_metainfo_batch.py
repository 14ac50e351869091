"""krk_metainfo_batch_dev (device.metainfo_batch): Generator.Generate over device-resident
blobs -- piece sums + InfoHash per blob, pipelined in groups -- against the oracle's
calcPieceSums (core/metainfo.go:157-179) and bencode + SHA-1 InfoHash
(core/metainfo.go:37-44), on seeded synthetic blobs of mixed sizes."""
import numpy as np
import pytest

from kraken_amd import device as D

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lengths,piece", [
    ([0, 1, 4095, 4096, 4097, 10 * 4096 + 3], 4096),       # empty blob, exact and ragged pieces
    ([1 << 20], 1 << 18),                                   # one blob: one group
    ([(i * 7919) % 300_000 + 1 for i in range(37)], 1 << 16),  # more blobs than groups
])
def test_metainfo_batch_matches_oracle(gpu, orc, lengths, piece):
    ids = [4000 + i for i in range(len(lengths))]
    arena = D.BlobArena(lengths, piece, blob_ids=ids)
    out = D.BatchOutputs(arena)
    names = [f"{i:064x}" for i in ids]
    sums_h = np.zeros(max(arena.total_pieces, 1), dtype=np.uint32)
    ih = D.metainfo_batch(arena, out, names, sums_h)
    dev = out.sums.to_host(np.uint32, max(arena.total_pieces, 1))
    assert np.array_equal(dev[:arena.total_pieces], sums_h[:arena.total_pieces])
    for k, L in enumerate(lengths):
        _, want = orc.calc_piece_sums(orc.synth(ids[k], L), piece)
        want = [int(x) for x in want]
        o, c = int(arena.sums_off[k]), int(arena.n_pieces[k])
        assert sums_h[o:o + c].tolist() == want
        assert bytes(ih[k]) == orc.info_hash(piece, want, names[k], L)


def test_metainfo_batch_rejects_bad_piece_length(gpu):
    arena = D.BlobArena([100], 64)
    out = D.BatchOutputs(arena)
    arena.piece_lengths[:] = 0
    arena._structs = None  # rebuild the krk_blob array with the bad piece length
    with pytest.raises(Exception, match="piece length must be positive"):
        D.metainfo_batch(arena, out, ["0" * 64], np.zeros(4, np.uint32))


def test_c5_regen_at_config_law(gpu, orc):
    """config C5's regen batch at its own law -- 1,000 blobs of
    log-uniform sizes in [0, 1 GiB) (bench.py c5regen_lengths, ~52 GB in HBM) with the
    piece-length table of lib/metainfogen/config_test.go:26-30 ({0: 1MB, 2GB: 4MB,
    4GB: 8MB}: every blob < 2 GB takes 1 MiB pieces) through krk_metainfo_batch_dev.
    Every blob's InfoHash is checked against the oracle's bencode + SHA-1 over its sums,
    and the sums of sampled blobs (the shortest, the longest, the median, 5 seeded
    others) against the oracle's calcPieceSums (core/metainfo.go:157-179)."""
    import bench
    from kraken_amd import metainfogen
    lens = bench.c5regen_lengths(1000)
    cfg = metainfogen.newPieceLengthConfig({0: 1 << 20, 2 << 30: 4 << 20, 4 << 30: 8 << 20})
    pls = {cfg.get(L) for L in lens}
    assert pls == {1 << 20}
    P = pls.pop()
    ids = [(1 << 40) + i for i in range(len(lens))]
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    names = [f"{(i * 0x9E3779B97F4A7C15) & ((1 << 64) - 1):016x}" * 4 for i in ids]
    sums_h = np.zeros(max(arena.total_pieces, 1), dtype=np.uint32)
    ih = D.metainfo_batch(arena, out, names, sums_h)
    L = np.asarray(lens)
    assert L.max() > (1 << 30) - (64 << 20) and L.min() < 4096 and arena.total_pieces > 40_000
    for k, n in enumerate(lens):
        o, c = int(arena.sums_off[k]), int(arena.n_pieces[k])
        assert c == -(-n // P)
        assert bytes(ih[k]) == orc.info_hash(P, sums_h[o:o + c], names[k], n), k
    rng = np.random.default_rng(0xC5)
    order = np.argsort(L, kind="stable")
    picks = sorted({int(L.argmin()), int(L.argmax()), int(order[len(L) // 2])} |
                   {int(x) for x in rng.choice(len(L), 5, replace=False)})
    for k in picks:
        _, want = orc.calc_piece_sums(orc.synth(ids[k], lens[k]), P)
        o, c = int(arena.sums_off[k]), int(arena.n_pieces[k])
        assert np.array_equal(sums_h[o:o + c], np.asarray(want, dtype=np.uint32)), k
