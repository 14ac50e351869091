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
