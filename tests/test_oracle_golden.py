"""Pins the CPU oracle (test infrastructure) before anything is checked against it:
the reference's own known-answer tests plus golden vectors produced by
independent implementations (tests/golden/gen_golden.py)."""
import hashlib
import json
import math
import os
import struct
import zlib

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def test_reference_kats(orc):
    k = GOLD["kat"]
    ih = k["info_hash"]
    assert orc.info_hash(ih["piece_length"], ih["piece_sums"], ih["name"], ih["length"]).hex() == ih["expected"]
    assert orc.sha256(k["sha256_test"]["input"].encode()).hex() == k["sha256_test"]["expected"]
    assert "sha256:" + orc.sha256(b"").hex() == k["digest_empty_tar"]
    assert orc.crc32(k["crc32_check"]["input"].encode()) == k["crc32_check"]["expected"]
    for size, pl, i, want in k["get_piece_length"]:
        n = -(-size // pl)
        assert orc.get_piece_length(size, pl, n, i) == want
    rng = dict((a, b) for a, b in k["piece_length_ranges"]["ranges"])
    for size, want in k["piece_length_ranges"]["cases"]:
        assert orc.piece_length_for_size(rng, size) == want
    for s, h in k["murmur3_h1"]:
        assert orc.murmur3_h1(s.encode()) == int(h, 16)


def test_survey_sanity_vector(orc):
    """labels dummy-origin-master0{1,2,3}-zone2:80, weight 100."""
    labels = [f"dummy-origin-master0{i}-zone2:80" for i in (1, 2, 3)]
    h1 = [orc.murmur3_h1(bytes.fromhex("e3b0") + l.encode()) for l in labels]
    assert h1 == [0x826B41F830434FBC, 0xBB8FB798DBB4FA8A, 0x85319F9780C10BFC]
    assert orc.hrw_ordered("e3b0", labels, [100] * 3) == [2, 1, 0]
    assert orc.hrw_ordered("0000", labels, [100] * 3) == [0, 2, 1]
    assert orc.hrw_ordered("ffff", labels, [100] * 3) == [0, 2, 1]


def test_rehash_property(orc):
    """lib/hrw/rendezvous_test.go:59-98: 2^53..2^63 have zero low 53 bits -> 0.0
    without a hasher, non-zero (finite log) after the one-time rehash."""
    for s in GOLD["kat"]["rehash_inputs"]:
        v = int(s)
        assert orc.uint64_to_float64(v, rehash=False) == 0.0
        f = orc.uint64_to_float64(v, rehash=True)
        assert f != 0.0 and math.isfinite(math.log(f))


def test_synth_spec(orc):
    from tests.golden.gen_golden import synth
    for idx, L, var in [(0, 0, 0), (1, 1, 0), (2, 13, 0), (3, 4096 + 5, 1), (123456789, 100000, 0)]:
        assert orc.synth(idx, L, variant=var).tobytes() == synth(idx, L, var)
    # offsets inside a blob
    full = synth(77, 1000)
    assert orc.synth(77, 300, offset=123).tobytes() == full[123:423]


def test_piece_sums_golden(orc):
    from tests.golden.gen_golden import synth
    for c in GOLD["pieces"]:
        data = synth(c["blob"], c["length"], c["variant"])
        length, sums = orc.calc_piece_sums(data, c["piece_length"])
        assert length == c["length"] and sums.tolist() == c["sums"], c["blob"]
        assert orc.sha256(data).hex() == c["sha256"]
        assert orc.info_hash(c["piece_length"], sums, c["sha256"], c["length"]).hex() == c["info_hash"]
    for c in GOLD["big"]:
        data = synth(c["blob"], c["length"])
        _, sums = orc.calc_piece_sums(data, c["piece_length"])
        assert hashlib.sha256(sums.astype("<u4").tobytes()).hexdigest() == c["sums_sha256"]
        assert orc.sha256_shani(data).hex() == c["sha256"]


def test_piece_sums_edges(orc):
    with pytest.raises(ValueError, match="piece length must be positive"):
        orc.calc_piece_sums(b"abc", 0)
    assert orc.calc_piece_sums(b"", 4)[1].tolist() == []          # L = 0: no sums
    assert len(orc.calc_piece_sums(b"x" * 8, 4)[1]) == 2            # no empty trailing piece
    assert len(orc.calc_piece_sums(b"x" * 9, 4)[1]) == 3


def test_crc_and_sha_variants_agree(orc):
    rng = np.random.default_rng(0)
    for n in [0, 1, 15, 16, 63, 64, 65, 127, 128, 1000, 4096, 65537, 1 << 20]:
        d = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        assert orc.crc32(d) == zlib.crc32(d) == orc.crc32_clmul(d)
        assert orc.sha256(d) == hashlib.sha256(d).digest() == orc.sha256_shani(d)
        assert orc.sha1(d) == hashlib.sha1(d).digest()
    # crc32.Update continuation semantics
    a, b = b"hello ", b"world"
    assert orc.crc32(b, orc.crc32(a)) == zlib.crc32(a + b)


def test_bencode_layout(orc):
    b = orc.bencode_info(8, [1, 4294967295], "ab", 10)
    assert b == b"d6:Lengthi10e4:Name2:ab11:PieceLengthi8e9:PieceSumsli1ei4294967295eee"
    assert orc.bencode_info(4, [], "x", 0) == b"d6:Lengthi0e4:Name1:x11:PieceLengthi4e9:PieceSumslee"


def test_go_log_golden(orc):
    for xb, yb in GOLD["go_log"]:
        x = struct.unpack(">d", bytes.fromhex(xb))[0]
        assert struct.pack(">d", orc.go_log(x)).hex() == yb
    assert orc.go_log(0.0) == -math.inf and math.isnan(orc.go_log(-1.0))


def test_go_log_within_one_ulp_of_libm(orc):
    """An independent check on the Go math.Log restatement (the weighted HRW score's log,
    golden bits above come from the same restatement): Go's algorithm (FreeBSD e_log.c,
    documented error < 1 ulp) must agree with the C library's log to within one ulp on the
    score's domain s = val / 2^53 in (0, 1), and bit for bit on most inputs."""
    rng = np.random.default_rng(53)
    xs = np.concatenate([rng.random(20000), rng.random(2000) * 1e-12, [2.0 ** -53, 0.5, 1 - 2.0 ** -53]])
    exact = 0
    for x in xs:
        x = float(x)
        if x <= 0.0:
            continue
        g, c = orc.go_log(x), math.log(x)
        assert abs(g - c) <= math.ulp(c), (x, g, c)
        exact += g == c
    assert exact >= 0.9 * len(xs), exact  # 93.6 % of these inputs bit-equal


def test_hrw_golden(orc):
    for c in GOLD["hrw"]:
        order, scores = orc.hrw_ordered(c["key"], c["labels"], c["weights"], with_scores=True)
        assert order == c["order"], c["key"]
        assert [struct.pack(">d", s).hex() for s in scores] == c["score_bits"], c["key"]
    assert math.isnan(orc.hrw_score("zz", "a", 100))


def test_ring_golden(orc):
    for c in GOLD["ring"]:
        key = c["digest"][:4]  # ShardID (core/digest.go:148-150)
        order = orc.hrw_ordered(key, c["labels"], [100] * len(c["labels"]))
        assert orc.ring_locations(order, c["healthy"], c["max_replica"]) == c["locations"]


def test_baseline_runner_outputs(orc):
    """The timed CPU baseline computes the same products as the restatement."""
    lens = [0, 1000, (1 << 20) + 3, 3 << 20]
    t, dg, (sums, off) = orc.baseline_run(list(range(4)), lens, 1 << 20, threads=2, fast=True,
                                          want_outputs=True)
    assert t >= 0
    for i, L in enumerate(lens):
        data = orc.synth(i, L)
        assert bytes(dg[i]) == hashlib.sha256(data.tobytes()).digest()
        ref = orc.calc_piece_sums(data, 1 << 20)[1]
        assert sums[int(off[i]):int(off[i]) + len(ref)].tolist() == ref.tolist()


def test_crc_bufs_matches_zlib(orc):
    """The same-buffer CPU leg (one CRC per caller buffer, bench f1verify / C4 A/B) is zlib's
    crc32 of each buffer, empty ones included."""
    import zlib
    rng = np.random.default_rng(6)
    bufs = [rng.integers(0, 256, L, dtype=np.uint8) for L in (0, 1, 32767, 32768, 32769, (1 << 20) + 5)]
    t, sums = orc.crc_bufs([b.ctypes.data for b in bufs], [b.size for b in bufs], 3)
    assert t >= 0
    assert sums.tolist() == [zlib.crc32(b.tobytes()) for b in bufs]


def test_baseline_files_matches_zlib(orc, tmp_path):
    """The files CPU baseline (the reference's Generate over cache files: calcPieceSums over
    the file reader in 32 KiB reads) gives zlib's piece sums, and fails on a short file."""
    import zlib
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in (0, 1, 32769, (1 << 20) + 3, 5 << 20)]
    paths = []
    for i, x in enumerate(datas):
        p = tmp_path / f"f{i}"
        p.write_bytes(x)
        paths.append(str(p))
    P = 1 << 20
    _, sums, off = orc.baseline_files(paths, [len(x) for x in datas], P, 3)
    for i, x in enumerate(datas):
        assert list(sums[int(off[i]):int(off[i + 1])]) == [zlib.crc32(x[k:k + P]) for k in range(0, len(x), P)]
    with pytest.raises(OSError):
        orc.baseline_files(paths[-1:], [len(datas[-1]) + 1], P, 1)
    # with the upload verify pass: the digests are hashlib's
    _, sums2, _, dg = orc.baseline_files(paths, [len(x) for x in datas], P, 2, passes=3)
    assert np.array_equal(sums2, sums)
    assert [bytes(d) for d in dg] == [hashlib.sha256(x).digest() for x in datas]


def test_oracle_owner_table_is_the_per_key_oracle():
    """orc_ring_owner_table (the exhaustive checker of the device owner tables) is the
    per-key restatement looped over all 65,536 ShardIDs: rows sampled against
    orc_hrw_ordered + orc_ring_locations, and SURVEY.md 8(c)'s sanity vector (labels
    dummy-origin-master0{1,2,3}-zone2:80: e3b0 -> 03, 02, 01; 0000 and ffff -> 01, 03, 02)."""
    import numpy as np

    from oracle import oracle as O
    labels = [f"dummy-origin-master0{i}-zone2:80" for i in (1, 2, 3)]
    locs, counts = O.ring_owner_table(labels, [100] * 3, np.ones(3, np.uint8), 3)
    assert locs[0xE3B0].tolist() == [2, 1, 0] and locs[0].tolist() == [0, 2, 1] and locs[0xFFFF].tolist() == [0, 2, 1]
    assert (counts == 3).all()
    rng = np.random.default_rng(5)
    for N, R in ((5, 2), (16, 3)):
        labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(N)]
        healthy = (rng.random(N) < 0.75).astype(np.uint8)
        locs, counts = O.ring_owner_table(labels, [100] * N, healthy, R)
        for shard in list(range(0, 65536, 1021)) + [65535]:
            ref = O.ring_locations(O.hrw_ordered(f"{shard:04x}", labels, [100] * N), healthy, R)
            assert locs[shard, :counts[shard]].tolist() == ref and (locs[shard, counts[shard]:] == -1).all()
