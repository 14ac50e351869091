"""Host-side logic of the mirror API (no GPU): digest parsing/validation, InfoHash
hex, MetaInfo JSON, metainfogen config -- with the reference's error strings."""
import os
import numpy as np
import pytest

from kraken_amd import core, hrw, metainfogen


def test_digest_parse_and_validate():
    h = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    d = core.NewSHA256DigestFromHex(h)
    assert d.String() == core.DigestEmptyTar and d.Algo() == "sha256" and d.ShardID() == "e3b0"
    assert core.ParseSHA256Digest(core.DigestEmptyTar) == d
    with pytest.raises(ValueError, match="invalid sha256: expected 64 characters"):
        core.NewSHA256DigestFromHex("abc")
    with pytest.raises(ValueError, match="invalid sha256: hex"):
        core.NewSHA256DigestFromHex("z" * 64)
    with pytest.raises(ValueError, match="invalid digest: empty"):
        core.ParseSHA256Digest("")
    with pytest.raises(ValueError, match="expected '<algo>:<hex>'"):
        core.ParseSHA256Digest("sha256")
    with pytest.raises(ValueError, match="invalid digest algo"):
        core.ParseSHA256Digest("md5:" + h)


def test_infohash_hex():
    ih = core.NewInfoHashFromHex("85b978c4377625b3963df406d0dd3a1da5a7d9c3")
    assert ih.Hex() == "85b978c4377625b3963df406d0dd3a1da5a7d9c3"
    with pytest.raises(ValueError, match="expected 40 characters"):
        core.NewInfoHashFromHex("00")


def test_metainfo_backwards_compatibility_kat():
    """core/metainfo_test.go:61-76 (production agent metainfo -> same info hash)."""
    raw = (b'{"Info":{"PieceLength":4194304,"PieceSums":[2131691452],"Name":'
           b'"289314c356bc2a19802c3e31505506db30ea81a0bcaea4ec3e079524c8ac3cf5","Length":236},'
           b'"Announce":"","AnnounceList":null,"CreationDate":0,"Comment":"","CreatedBy":""}')
    mi = core.DeserializeMetaInfo(raw)
    assert mi.InfoHash() == core.NewInfoHashFromHex("85b978c4377625b3963df406d0dd3a1da5a7d9c3")
    assert mi.NumPieces() == 1 and mi.GetPieceLength(0) == 236 and mi.GetPieceLength(1) == 0
    back = core.DeserializeMetaInfo(mi.Serialize())
    assert back.InfoHash() == mi.InfoHash()


def test_metainfo_serialize_bytes_pinned_by_fixture():
    """Serialize (core/metainfo.go:131-134, json.Marshal of
    metaInfoJSON{info}) emits exactly {"Info": <the fixture's Info object>} for the
    production metainfo of core/metainfo_test.go:68 -- field order PieceLength,
    PieceSums, Name, Length, no spaces -- whether the MetaInfo was deserialized from the
    fixture or built from its fields."""
    info = (b'{"PieceLength":4194304,"PieceSums":[2131691452],"Name":'
            b'"289314c356bc2a19802c3e31505506db30ea81a0bcaea4ec3e079524c8ac3cf5","Length":236}')
    raw = b'{"Info":' + info + b',"Announce":"","AnnounceList":null,"CreationDate":0,"Comment":"","CreatedBy":""}'
    assert core.DeserializeMetaInfo(raw).Serialize() == b'{"Info":' + info + b'}'
    name = "289314c356bc2a19802c3e31505506db30ea81a0bcaea4ec3e079524c8ac3cf5"
    d = core.NewSHA256DigestFromHex(name)
    ih = core.NewInfoHashFromHex("85b978c4377625b3963df406d0dd3a1da5a7d9c3")
    built = core.MetaInfo(4194304, np.array([2131691452], dtype=np.uint32), name, 236, d, ih)
    assert built.Serialize() == b'{"Info":' + info + b'}'
    # nil PieceSums (a zero-length blob: calcPieceSums returns nil) marshals as null
    empty = core.MetaInfo(4194304, None, name, 0, d, ih)
    assert empty.Serialize() == (b'{"Info":{"PieceLength":4194304,"PieceSums":null,"Name":"' + name.encode() +
                                 b'","Length":0}}')


def test_deserialize_follows_encoding_json():
    """encoding/json rules for metaInfoJSON -- the exact key wins over a
    case-folded one and a later duplicate over an earlier one; null leaves an int64 /
    string field at its value and sets the slice to nil; type and range errors are
    "cannot unmarshal <kind> into Go struct field info.<Field> of type <T>"."""
    name = "289314c356bc2a19802c3e31505506db30ea81a0bcaea4ec3e079524c8ac3cf5"

    def mk(fields: str) -> bytes:
        return ('{"Info":{' + fields + '}}').encode()

    base = f'"PieceLength":4194304,"PieceSums":[2131691452],"Name":"{name}"'
    mi = core.DeserializeMetaInfo(mk(base + ',"Length":236'))
    assert mi.InfoHash().Hex() == "85b978c4377625b3963df406d0dd3a1da5a7d9c3"
    # case-insensitive key, later duplicate wins, null keeps the value
    assert core.DeserializeMetaInfo(mk(base + ',"length":5,"Length":236')).Length() == 236
    assert core.DeserializeMetaInfo(mk(base + ',"Length":236,"LENGTH":7')).Length() == 7
    assert core.DeserializeMetaInfo(mk(base + ',"Length":236,"Length":null')).Length() == 236
    assert core.DeserializeMetaInfo(mk(f'"PieceLength":4,"PieceSums":null,"Name":"{name}"')).PieceSums().size == 0
    cases = [
        (',"Length":9223372036854775808', "cannot unmarshal number 9223372036854775808 into Go struct field "
                                          "info.Length of type int64"),
        (',"Length":1.5', "cannot unmarshal number 1.5 into Go struct field info.Length of type int64"),
        (',"Length":"236"', "cannot unmarshal string into Go struct field info.Length of type int64"),
        (',"Length":true', "cannot unmarshal bool into Go struct field info.Length of type int64"),
    ]
    for extra, msg in cases:
        with pytest.raises(ValueError) as ei:
            core.DeserializeMetaInfo(mk(base + extra))
        assert str(ei.value) == "json: " + msg, extra
    bad_sums = [('[4294967296]', "number 4294967296", "uint32"), ('[-1]', "number -1", "uint32"),
                ('["x"]', "string", "uint32"), ('{"a":1}', "object", "[]uint32"), ('7', "number 7", "[]uint32")]
    for arr, what, typ in bad_sums:
        with pytest.raises(ValueError) as ei:
            core.DeserializeMetaInfo(mk(f'"PieceLength":4,"PieceSums":{arr},"Name":"{name}","Length":1'))
        assert str(ei.value) == f"json: cannot unmarshal {what} into Go struct field info.PieceSums of type {typ}"
    with pytest.raises(ValueError, match="json: cannot unmarshal array into Go value of type core.metaInfoJSON"):
        core.DeserializeMetaInfo(b"[]")
    with pytest.raises(ValueError, match="parse name"):
        core.DeserializeMetaInfo(b'{"Info":null}')


def test_metainfo_serialization_limit():
    """core/metainfo_test.go:78-120: 100 GB / 2 MB pieces stays under 512 MB of JSON."""
    n = (100 << 30) // (2 << 20)
    sums = np.random.default_rng(0).integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32)
    mi = core.MetaInfo(2 << 20, sums, "6422b52513a39399598494bdb7471211890cd13c271fb5c11c5ba6538ed7578c",
                       100 << 30, None, None)
    assert len(mi.Serialize()) < 512 << 20


def test_deserialize_errors():
    with pytest.raises(ValueError, match="json"):
        core.DeserializeMetaInfo(b"{")
    with pytest.raises(ValueError, match="parse name"):
        core.DeserializeMetaInfo(b'{"Info":{"PieceLength":1,"PieceSums":[],"Name":"x","Length":0}}')


def test_piece_length_config():
    """lib/metainfogen/config_test.go:23-38."""
    c = metainfogen.newPieceLengthConfig({0: 1 << 20, 2 << 30: 4 << 20, 4 << 30: 8 << 20})
    assert c.get(1 << 30) == 1 << 20
    assert c.get(2 << 30) == 4 << 20
    assert c.get(3 << 30) == 4 << 20
    assert c.get(4 << 30) == 8 << 20
    assert c.get(8 << 30) == 8 << 20
    with pytest.raises(ValueError, match="no piece lengths configured"):
        metainfogen.newPieceLengthConfig({})
    with pytest.raises(ValueError, match="piece length config: no piece lengths configured"):
        metainfogen.New({}, None)


def test_score_function_float_precision():
    """lib/hrw/rendezvous_test.go:30-57 (TestScoreFunctionFloatPrecision)."""
    import math
    from kraken_amd import hrw
    for idx, bl in enumerate((8, 16, 32)):
        for si, f in enumerate((hrw.BigIntToFloat64, hrw.UInt64ToFloat64)):
            if idx > 0 and si > 0:
                continue
            v = f(b"\x00" * (bl - 1) + b"\x01", b"\xff" * bl, None)
            assert v != 0.0 and math.isfinite(math.log(v))


def test_bigint_to_float64_rounding():
    """BigIntToFloat64 = round53(round53(h) / max): exact cases and correct rounding."""
    from fractions import Fraction
    from kraken_amd import hrw
    M8 = b"\xff" * 8
    assert hrw.BigIntToFloat64((1 << 63).to_bytes(8, "big"), M8) == 0.5
    assert hrw.BigIntToFloat64(b"\xff" * 8, M8) == 1.0
    assert hrw.BigIntToFloat64(b"\x00" * 8, M8) == 0.0
    rng = np.random.default_rng(7)
    for bl in (8, 16, 32):
        M = (1 << (8 * bl)) - 1
        for _ in range(200):
            h = int.from_bytes(rng.bytes(bl), "big")
            got = hrw.BigIntToFloat64(h.to_bytes(bl, "big"), M.to_bytes(bl, "big"))
            h53 = hrw._round_prec(h, 53)
            assert h53.bit_length() <= max(53, h.bit_length() + 1)
            exact = Fraction(h53, M)
            # nearest double: no double strictly closer than `got`
            lo, hi = np.nextafter(got, 0.0), np.nextafter(got, 2.0)
            assert abs(Fraction(got) - exact) <= abs(Fraction(float(lo)) - exact)
            assert abs(Fraction(got) - exact) <= abs(Fraction(float(hi)) - exact)


def test_uint64_to_float64_host_matches_oracle(orc):
    """rendezvous.go:99-118: host helper == oracle restatement, incl. the rehash rule."""
    from kraken_amd import hrw
    rh = lambda b: orc.murmur3_h1(b).to_bytes(8, "big")
    vals = [1, 2, (1 << 53) - 1, 1 << 53, 1 << 60, (1 << 64) - 1, 0x123456789ABCDEF0] + [1 << k for k in range(53, 64)]
    for v in vals:
        b = v.to_bytes(8, "big")
        assert hrw.UInt64ToFloat64(b, rehash=rh) == orc.uint64_to_float64(v, rehash=True), hex(v)
        assert hrw.UInt64ToFloat64(b) == orc.uint64_to_float64(v, rehash=False), hex(v)


def test_dircas_layout_and_list_names(tmp_path):
    """DirCAS follows casFileEntryFactory.GetRelativePath (lib/store/base/file_entry.go:176-189)."""
    from kraken_amd import metainfogen
    cas = metainfogen.DirCAS(str(tmp_path))
    name = "07123e1f482356c415f684407a3b8723e10b2cbbc0b8fcd6282c49d37c9c1abc"  # the reference's example
    assert cas._dir(name) == str(tmp_path / "07" / "12" / name)
    names = [name, "ff" * 32, "00ab" + "1" * 60]
    for n in names:
        os.makedirs(cas._dir(n))
        open(os.path.join(cas._dir(n), "data"), "wb").close()
    os.makedirs(tmp_path / "07" / "12" / "stray")  # no data file: not a blob
    assert cas.ListNames() == sorted(names)
    assert metainfogen._parse_config("0:4194304,2147483648:8388608") == {0: 4194304, 2147483648: 8388608}


def test_generate_error_wrapping(tmp_path):
    """lib/metainfogen/generator.go:41-58 error prefixes, on the paths that fail before
    any device work: a missing cache file and an unreadable one."""
    cas = metainfogen.DirCAS(str(tmp_path))
    g = metainfogen.New({0: 1 << 20}, cas)
    d = core.NewSHA256DigestFromHex("ab" * 32)
    with pytest.raises(IOError, match=r"^cache stat: "):
        g.Generate(d)

    class Unreadable(metainfogen.DirCAS):
        def GetCacheFileReader(self, hex_):
            raise OSError("permission denied")

    os.makedirs(cas._dir(d.Hex()))
    open(os.path.join(cas._dir(d.Hex()), "data"), "wb").close()
    with pytest.raises(IOError, match=r"^get cache file: permission denied"):
        metainfogen.New({0: 1 << 20}, Unreadable(str(tmp_path))).Generate(d)


def _plan_checks(lens, W, cap):
    from kraken_amd.windowed import window_plan
    wins = window_plan(lens, W, cap)
    L = np.asarray(lens, dtype=np.uint64)
    covered = np.zeros(len(lens), dtype=np.uint64)
    started = {}
    for k, (blobs, offs, take) in enumerate(wins):
        assert 0 < blobs.size <= max(1, min(cap, len(lens)))
        assert np.array_equal(offs, covered[blobs])  # each chunk continues its blob
        assert np.all(take > 0)
        # every chunk but a blob's last is a multiple of 64 (whole SHA-256 blocks)
        last = offs + take == L[blobs]
        assert np.all(take[~last] % 64 == 0)
        covered[blobs] += take
        for b in blobs.tolist():
            started.setdefault(b, k)
    assert np.array_equal(covered, L)  # every byte exactly once
    return wins, started


def test_c3_window_plan_admits_longest_first_under_cap():
    """kraken_amd.windowed.window_plan: bytes covered exactly once, <= cap live blobs a window,
    and a blob never starts after a shorter one."""
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(1, 5000, size=300)] + [0 + 64, 12_345, 64 * 1000]
    W, cap = 64 * 1024, 37
    wins, started = _plan_checks(lens, W, cap)
    order = sorted(range(len(lens)), key=lambda i: (-lens[i], i))
    starts = [started[i] for i in order]
    assert starts == sorted(starts)
    assert started[order[0]] == 0


def test_c3_window_plan_no_cap_and_single_blob():
    lens = [1000, 64, 129, 5000]
    wins, started = _plan_checks(lens, 4096, len(lens))
    assert all(v == 0 for v in started.values())  # all live from window 0
    wins, _ = _plan_checks([10**6], 1 << 16, 16384)
    assert len(wins) == -(-10**6 // (1 << 16))


def test_validate_sha256_go_errors():
    """core/digest.go:152-161 via hex.DecodeString: a trailing newline is an invalid
    byte (the length counts bytes, as Go's len does)."""
    good = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    core.ValidateSHA256(good)
    core.ValidateSHA256(good.upper())
    with pytest.raises(ValueError, match=r"^hex: encoding/hex: invalid byte: U\+000A$"):
        core.ValidateSHA256(good[:63] + "\n")
    with pytest.raises(ValueError, match=r"^hex: encoding/hex: invalid byte: U\+0067 'g'$"):
        core.ValidateSHA256("g" + good[1:])
    with pytest.raises(ValueError, match=r'^expected 64 characters, got 2 from "ab"$'):
        core.ValidateSHA256("ab")
    with pytest.raises(ValueError, match=r"^invalid sha256: expected 64 characters"):
        core.NewSHA256DigestFromHex(good + "\n")


def test_deserialize_partial_sidecar_zero_values():
    """json.Unmarshal fills absent fields (and a null Info) with zero values, so a
    truncated or partial _torrentmeta fails on the name, like the reference."""
    for raw in (b'{"Info":null}', b'{}', b'{"Info":{"PieceLength":4}}', b'null',
                b'{"Info":{"PieceSums":[1,2],"Length":3}}'):
        with pytest.raises(ValueError, match=r'^parse name: invalid sha256: expected 64 characters, got 0 from ""$'):
            core.DeserializeMetaInfo(raw)
    with pytest.raises(ValueError, match=r"^json: "):
        core.DeserializeMetaInfo(b'{"Info":{"PieceLength":"x"}}')
    with pytest.raises(ValueError, match=r"^json: "):
        core.DeserializeMetaInfo(b'[1]')


def test_get_ordered_nodes_negative_n():
    """GetOrderedNodes(key, n < 0): the reference panics on nodes[:n]; never reaches the device."""
    rh = hrw.NewRendezvousHash()
    rh.AddNode("a", 100)
    with pytest.raises(ValueError):
        rh.GetOrderedNodes("00ff", -1)
    with pytest.raises(ValueError):
        rh.GetOrderedNodesBatch(["00ff"], -3)


def test_cas_volume_symlink_refuses_non_links(tmp_path):
    """createOrUpdateSymlink (lib/store/utils.go:25-47): a regular file or a real
    directory at <dir>/<subdir> is an error and stays in place (initCASVolumes wraps
    it as "symlink to volume: ...")."""
    from kraken_amd import castore
    vol = tmp_path / "vol"
    vol.mkdir()
    d = tmp_path / "cas"
    d.mkdir()
    (d / "00").write_bytes(b"user data")
    with pytest.raises(OSError):
        castore._create_or_update_symlink(str(vol / "cas" / "00"), str(d / "00"))
    assert (d / "00").read_bytes() == b"user data"
    (d / "01").mkdir()
    with pytest.raises(OSError):
        castore._create_or_update_symlink(str(vol / "x"), str(d / "01"))
    assert (d / "01").is_dir() and not (d / "01").is_symlink()
    # existing link to another place is replaced; a missing target is created
    os.symlink(str(vol), str(d / "02"))
    castore._create_or_update_symlink(str(vol / "cas" / "02"), str(d / "02"))
    assert os.readlink(str(d / "02")) == str(vol / "cas" / "02")
    castore._create_or_update_symlink(str(vol / "cas" / "03"), str(d / "03"))
    assert os.readlink(str(d / "03")) == str(vol / "cas" / "03")
