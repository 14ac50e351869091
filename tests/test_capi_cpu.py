"""CPU-only checks of the C ABI boundary: the library loads, exports every symbol
include/kraken_hip.h declares, the Python binding covers all of them, and the
host-side entry points (no GPU) agree with the oracle.  Device entry points must
fail loudly (KRK_ENODEV), never fall back to the CPU."""
import ctypes as C
import subprocess

import numpy as np
import pytest

from kraken_amd import _capi
from kraken_amd._capi import KRK_ENODEV, check, lib


def test_library_exports_every_declared_symbol():
    declared = _capi.declared_symbols()
    assert len(declared) >= 38
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)
    assert set(declared) == set(lib._krk_sigs), set(declared) ^ set(lib._krk_sigs)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _capi.LIB_PATH], capture_output=True,
                         text=True)
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_library_does_not_link_the_oracle():
    out = subprocess.run(["ldd", _capi.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    assert b"orc_" not in open(_capi.LIB_PATH, "rb").read()


def test_version_and_errors():
    assert lib.krk_version().startswith(b"kraken_amd")
    assert lib.krk_last_error() is not None


def test_info_hash_and_bencode_match_oracle(orc):
    rng = np.random.default_rng(2)
    for n in [0, 1, 7, 1000]:
        sums = rng.integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32)
        name = rng.bytes(32).hex()
        L = int(rng.integers(0, 1 << 40))
        P = int(rng.integers(1, 1 << 30))
        out = (C.c_uint8 * 20)()
        sp = sums.ctypes.data_as(C.POINTER(C.c_uint32)) if n else None
        check(lib.krk_info_hash(P, sp, n, name.encode(), 64, L, out))
        assert bytes(out) == orc.info_hash(P, sums, name, L)
        w = C.c_uint64()
        check(lib.krk_bencode_info(P, sp, n, name.encode(), 64, L, None, 0, C.byref(w)))
        buf = (C.c_uint8 * w.value)()
        check(lib.krk_bencode_info(P, sp, n, name.encode(), 64, L, buf, w.value, C.byref(w)))
        assert bytes(buf) == orc.bencode_info(P, sums, name, L)
    small = (C.c_uint8 * 4)()
    assert lib.krk_bencode_info(1, None, 0, b"x", 1, 0, small, 4, C.byref(w)) == _capi.KRK_ERANGE


def test_num_pieces_and_piece_length_config(orc):
    for L, P in [(0, 1), (1, 1), (10, 3), (8, 2), (1 << 30, 4 << 20), ((1 << 30) + 1, 4 << 20)]:
        assert lib.krk_num_pieces(L, P) == -(-L // P)
    assert lib.krk_num_pieces(10, 0) == 0
    t = np.array([0, 2 << 30, 4 << 30], dtype=np.int64)
    l = np.array([1 << 20, 4 << 20, 8 << 20], dtype=np.int64)
    for size in [0, 1 << 30, 2 << 30, 3 << 30, 4 << 30, 8 << 30]:
        got = lib.krk_piece_length_for_size(t.ctypes.data_as(C.POINTER(C.c_int64)),
                                             l.ctypes.data_as(C.POINTER(C.c_int64)), 3, size)
        assert got == orc.piece_length_for_size({0: 1 << 20, 2 << 30: 4 << 20, 4 << 30: 8 << 20}, size)


def test_device_entry_points_fail_loudly_without_gpu():
    """Device entry points and the GPU placements are KRK_ENODEV without a gfx950 device:
    nothing falls back to the CPU."""
    n = C.c_int(-1)
    check(lib.krk_device_count(C.byref(n)))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    assert lib.krk_digester_new_on(_capi.KRK_PLACE_GPU, C.byref(h)) == KRK_ENODEV
    assert lib.krk_piece_stream_begin_on(_capi.KRK_PLACE_GPU, 4, C.byref(h)) == KRK_ENODEV
    out = C.c_uint32()
    big = b"x" * (1 << 20)
    assert lib.krk_crc32_update_on(_capi.KRK_PLACE_GPU, 0, big, len(big), C.byref(out)) == KRK_ENODEV
    assert b"no HIP device" in lib.krk_last_error()
    blob = (_capi.krk_blob * 1)(_capi.krk_blob(None, 0, 4, 0))
    assert lib.krk_metainfo_digest_host(blob, 1, None, (C.c_uint8 * 32)()) == KRK_ENODEV
    assert lib.krk_metainfo_digest_host_multi(blob, 1, None, (C.c_uint8 * 32)()) == KRK_ENODEV
    assert lib.krk_piece_sums_dev(blob, 1, None, None) == KRK_ENODEV
    # a process-wide GPU setting makes AUTO a forced GPU placement, which has no fallback
    check(lib.krk_set_crc_placement(_capi.KRK_PLACE_GPU))
    try:
        assert lib.krk_piece_stream_begin(4, C.byref(h)) == KRK_ENODEV
        assert lib.krk_crc32_update(0, big, len(big), C.byref(out)) == KRK_ENODEV
    finally:
        check(lib.krk_set_crc_placement(_capi.KRK_PLACE_AUTO))


def _ih(P, sums, name, L):
    out = (C.c_uint8 * 20)()
    s = np.ascontiguousarray(sums, dtype=np.uint32)
    check(lib.krk_info_hash(P, s.ctypes.data_as(C.POINTER(C.c_uint32)) if s.size else None, s.size,
                            name.encode(), len(name.encode()), L, out))
    return bytes(out)


def test_info_hash_reference_kat():
    """core/metainfo_test.go:61-76 through the C ABI (host bencode + SHA-1)."""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    k = gold["kat"]["info_hash"]
    assert _ih(k["piece_length"], k["piece_sums"], k["name"], k["length"]).hex() == k["expected"]


def test_info_hash_every_tail_length(orc):
    """Every bencode length residue mod 64 (the SHA-1 tail and two-block padding cases),
    large and negative integers, against the oracle's independent SHA-1 + bencode."""
    rng = np.random.default_rng(9)
    for n in list(range(0, 140)) + [999, 4096, 81920]:
        sums = rng.integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32)
        name = rng.bytes(int(rng.integers(0, 40))).hex()
        L = int(rng.integers(-(1 << 62), 1 << 62))
        P = int(rng.integers(1, 1 << 40))
        assert _ih(P, sums, name, L) == orc.info_hash(P, sums, name, L), n


_IH_SCRIPT = """
import sys, ctypes as C
import numpy as np
sys.path.insert(0, sys.argv[1])
from kraken_amd._capi import lib
rng = np.random.default_rng(3)
out = []
for n in range(0, 300, 7):
    s = rng.integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32)
    o = (C.c_uint8 * 20)()
    lib.krk_info_hash(12345, s.ctypes.data_as(C.POINTER(C.c_uint32)) if n else None, n, b"ab", 2, n, o)
    out.append(bytes(o).hex())
print(" ".join(out))
"""


def test_info_hash_sha_ni_matches_portable_sha1(tmp_path):
    """The SHA-NI compressor (when this CPU has it) and the portable one agree: the production
    library against the diag build with KRK_SHA1_PORTABLE=1 (an A/B switch production does
    not read, knobs.hpp)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "ih.py"
    f.write_text(_IH_SCRIPT)
    from tests.conftest import diag_lib
    runs = [subprocess.run([sys.executable, str(f), root], capture_output=True, text=True, env=env)
            for env in (dict(os.environ), {**os.environ, "KRK_SHA1_PORTABLE": "1", "KRK_LIB_PATH": diag_lib()})]
    assert all(r.returncode == 0 for r in runs), [r.stderr for r in runs]
    assert runs[0].stdout == runs[1].stdout and len(runs[0].stdout.split()) == 43


def test_info_hash_batch_matches_single(orc):
    from kraken_amd import core
    rng = np.random.default_rng(17)
    n = 300
    ns = rng.integers(0, 50, n)
    ns[::7] = 0
    sums = rng.integers(0, 2 ** 32, size=int(ns.sum()), dtype=np.uint64).astype(np.uint32)
    off = np.concatenate(([0], np.cumsum(ns)[:-1]))
    names = [rng.bytes(32).hex() if i % 5 else "" for i in range(n)]
    pls = rng.integers(1, 1 << 30, n)
    lens = rng.integers(0, 1 << 40, n)
    got = core._info_hash_batch(pls, sums, off, ns, names, lens)
    for i in range(n):
        s = sums[off[i]:off[i] + ns[i]]
        assert bytes(got[i]) == orc.info_hash(int(pls[i]), s, names[i], int(lens[i])), i


def test_production_library_has_no_diagnostic_kernels():
    """The timing diagnostics (wrong results by design) and the measured-but-unused
    layouts are compiled only into the KRK_DIAG build (make diag): the production .so
    carries exactly the production kernel instantiations."""
    out = subprocess.run(["nm", "-C", _capi.LIB_PATH], capture_output=True, text=True).stdout
    kern = sorted({l.split(" ", 2)[2] for l in out.splitlines() if "__device_stub__" in l})
    sha = [k for k in kern if "sha256" in k]
    crc = [k for k in kern if "crc_items_kernel" in k]
    assert sha and crc
    assert all(("sha256_ws_kernel<0," in k or "sha256_w8_kernel<0," in k) for k in sha), sha  # kTiming = 0 only
    assert not any("sha256_multi_kernel" in k for k in kern)
    # crc_items_kernel<R, RG, BLOCK, COAL, LOADONLY, PERM, NT>: strided, no load-only, no NT
    assert all(k.split("<")[1].startswith(("32, 4, 1024, false, false, 32, false",
                                           "32, 8, 1024, false, false, 32, false",
                                           "16, 4, 1024, false, false, 16, false")) for k in crc), crc
    assert b"KRK_SHA_VARIANT" not in open(_capi.LIB_PATH, "rb").read()


def test_host_crossover_primitives_match_hashlib_zlib():
    import hashlib
    import zlib
    rng = np.random.default_rng(11)
    for n in list(range(0, 200)) + [255, 256, 1023, 4096, 65535, 65536, (1 << 20) + 5]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        o = (C.c_uint8 * 32)()
        check(lib.krk_host_sha256(d, n, o))
        assert bytes(o) == hashlib.sha256(d).digest(), n
        seed = int(rng.integers(0, 2 ** 32))
        c = C.c_uint32()
        check(lib.krk_host_crc32_update(seed, d, n, C.byref(c)))
        assert c.value == zlib.crc32(d, seed), n


def test_host_crc_folding_paths_match_zlib():
    """The host CRC's folding loops -- AVX-512 VPCLMULQDQ (256 bytes an iteration, then 64-byte
    and 16-byte folds) where this CPU has it, the 128-bit PCLMUL loop otherwise -- at every
    length around their block edges and at unaligned addresses, against zlib."""
    import zlib
    rng = np.random.default_rng(12)
    buf = rng.integers(0, 256, (1 << 20) + 64, dtype=np.uint8)
    lens = [n for b in (64, 256, 512, 768, 4096) for n in range(b - 17, b + 18)]
    lens += [int(x) for x in rng.integers(0, 1 << 20, 64)]
    c = C.c_uint32()
    for n in lens:
        for off in (0, 3, 40):
            seed = int(rng.integers(0, 2 ** 32))
            check(lib.krk_host_crc32_update(seed, buf.ctypes.data + off, n, C.byref(c)))
            assert c.value == zlib.crc32(buf[off:off + n].tobytes(), seed), (n, off)


_HOST_SCRIPT = """
import sys, ctypes as C, numpy as np
sys.path.insert(0, sys.argv[1])
from kraken_amd._capi import lib
rng = np.random.default_rng(5)
out = []
for n in [0, 1, 63, 64, 65, 127, 128, 1000, 4096, 100003]:
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    o = (C.c_uint8 * 32)(); c = C.c_uint32()
    lib.krk_host_sha256(d, n, o); lib.krk_host_crc32_update(7, d, n, C.byref(c))
    out.append(bytes(o).hex() + "%08x" % c.value)
print(" ".join(out))
"""


def test_host_crossover_ni_matches_portable(tmp_path):
    """SHA-NI / PCLMULQDQ / VPCLMULQDQ routines (when this CPU has them) equal the portable
    ones (KRK_HOST_CRC_AVX512=0: the 128-bit PCLMUL loop): the production library against the
    diag build with those A/B switches set (production does not read them, knobs.hpp)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "h.py"
    f.write_text(_HOST_SCRIPT)
    from tests.conftest import diag_lib
    runs = [subprocess.run([sys.executable, str(f), root], capture_output=True, text=True,
                           env={**os.environ, **extra})
            for extra in ({}, {"KRK_LIB_PATH": diag_lib(), "KRK_HOST_PORTABLE": "1", "KRK_HOST_CRC_AVX512": "1"},
                          {"KRK_LIB_PATH": diag_lib(), "KRK_HOST_PORTABLE": "0", "KRK_HOST_CRC_AVX512": "0"})]
    assert all(r.returncode == 0 for r in runs), [r.stderr for r in runs]
    assert runs[0].stdout == runs[1].stdout == runs[2].stdout and len(runs[0].stdout.split()) == 10


def test_host_placements_work_without_a_device():
    """a host-placed Digester, piece stream and crc32.Update run the
    product's own SHA-NI / PCLMUL code (host_meta.cpp, not the oracle) and need no device;
    AUTO on a host without a gfx950 device is the host placement.  (On a GPU host the
    same calls place by the crossover, tests/test_gpu_crossover.py.)"""
    import hashlib
    import zlib
    n = C.c_int(-1)
    check(lib.krk_device_count(C.byref(n)))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    rng = np.random.default_rng(21)
    data = rng.integers(0, 256, (3 << 20) + 12345, dtype=np.uint8).tobytes()
    for p in (_capi.KRK_PLACE_AUTO, _capi.KRK_PLACE_HOST):
        h = C.c_void_p()
        check(lib.krk_digester_new_on(p, C.byref(h)))
        try:
            where = C.c_int(-1)
            check(lib.krk_digester_placement(h, C.byref(where)))
            assert where.value == _capi.KRK_PLACE_HOST
            for a in range(0, len(data), 1 << 19):  # io.Copy-like writes
                chunk = data[a:a + (1 << 19) - 7]
                check(lib.krk_digester_write(h, chunk, len(chunk)))
            o = (C.c_uint8 * 32)()
            check(lib.krk_digester_sum(h, o))
            seen = b"".join(data[a:a + (1 << 19) - 7] for a in range(0, len(data), 1 << 19))
            assert bytes(o) == hashlib.sha256(seen).digest()
        finally:
            lib.krk_digester_free(h)
        for P in (1, 7, 1 << 20):
            s = C.c_void_p()
            check(lib.krk_piece_stream_begin_on(p, P, C.byref(s)))
            try:
                where = C.c_int(-1)
                check(lib.krk_piece_stream_placement(s, C.byref(where)))
                assert where.value == _capi.KRK_PLACE_HOST
                blob = data[:200_001] if P < 8 else data
                step = 65_537
                for a in range(0, len(blob), step):
                    check(lib.krk_piece_stream_update(s, blob[a:a + step], len(blob[a:a + step])))
                ns, ln = C.c_uint64(), C.c_uint64()
                check(lib.krk_piece_stream_end(s, None, 0, C.byref(ns), C.byref(ln)))
                sums = (C.c_uint32 * ns.value)()
                check(lib.krk_piece_stream_end(s, sums, ns.value, C.byref(ns), C.byref(ln)))
                want = [zlib.crc32(blob[i:i + P]) for i in range(0, len(blob), P)]
                assert ln.value == len(blob) and list(sums) == want, P
            finally:
                lib.krk_piece_stream_free(s)
        out = C.c_uint32()
        check(lib.krk_crc32_update_on(p, 12345, data, len(data), C.byref(out)))
        assert out.value == zlib.crc32(data, 12345)
    out = C.c_uint32()
    check(lib.krk_crc32_update(7, data, len(data), C.byref(out)))  # AUTO, no device: host
    assert out.value == zlib.crc32(data, 7)
    h = C.c_void_p()
    assert lib.krk_digester_new_on(7, C.byref(h)) == _capi.KRK_EINVAL
    assert lib.krk_piece_stream_begin_on(1, 0, C.byref(h)) == _capi.KRK_EINVAL
    assert lib.krk_last_error() == b"piece length must be positive"


def test_host_crc_spans_on_the_pool_match_zlib():
    """Large host-placed writes are cut into spans that idle host-pool threads hash beside
    the caller (host_pool.cpp); the spans' CRCs recombine (GF(2) shift + xor) to exactly
    crc32.Update of the whole write, across piece ends and with seeds."""
    import zlib
    rng = np.random.default_rng(23)
    data = rng.integers(0, 256, (37 << 20) + 4321, dtype=np.uint8).tobytes()
    for seed in (0, 0xDEADBEEF):
        for n in (2 << 20, (2 << 20) + 1, (9 << 20) + 77, len(data)):
            out = C.c_uint32()
            check(lib.krk_crc32_update_on(_capi.KRK_PLACE_HOST, seed, data, n, C.byref(out)))
            assert out.value == zlib.crc32(data[:n], seed), (seed, n)
    for P in ((1 << 20) + 1, 4 << 20, 64 << 10, 3):
        s = C.c_void_p()
        check(lib.krk_piece_stream_begin_on(_capi.KRK_PLACE_HOST, P, C.byref(s)))
        try:
            blob = data if P >= (64 << 10) else data[:(3 << 20) + 1]
            pos = 0
            for step in [(4 << 20) + 3, 5, (2 << 20), (8 << 20) - 1] * 10:
                if pos >= len(blob):
                    break
                chunk = blob[pos:pos + step]
                check(lib.krk_piece_stream_update(s, chunk, len(chunk)))
                pos += len(chunk)
            rest = blob[pos:]
            if rest:
                check(lib.krk_piece_stream_update(s, rest, len(rest)))
            ns, ln = C.c_uint64(), C.c_uint64()
            check(lib.krk_piece_stream_end(s, None, 0, C.byref(ns), C.byref(ln)))
            sums = (C.c_uint32 * ns.value)()
            check(lib.krk_piece_stream_end(s, sums, ns.value, C.byref(ns), C.byref(ln)))
            assert ln.value == len(blob)
            assert list(sums) == [zlib.crc32(blob[i:i + P]) for i in range(0, len(blob), P)], P
        finally:
            lib.krk_piece_stream_free(s)


def test_offload_setting_defaults_to_auto():
    """the SHA-256 host offload is planner-gated AUTO by default."""
    t = C.c_int(99)
    check(lib.krk_sha_host_offload(C.byref(t)))
    assert t.value == _capi.KRK_OFFLOAD_AUTO == -1
    assert lib.krk_set_sha_host_offload(-2) == _capi.KRK_EINVAL
    check(lib.krk_set_sha_host_offload(0))
    check(lib.krk_sha_host_offload(C.byref(t)))
    assert t.value == 0
    check(lib.krk_set_sha_host_offload(_capi.KRK_OFFLOAD_AUTO))


def test_sha_offload_plan():
    """krk_sha_offload_plan (host offload of the longest SHA-256 chains): equal blobs
    stay on the GPU, a lone long blob goes to the host, a log-uniform batch hands over
    exactly its longest blobs and shortens its modelled makespan; threads = 0 is off."""
    from kraken_amd import device as D
    idx, g, h = D.sha_offload_plan([100 << 20] * 1000, 16)  # C2
    assert idx.size == 0 and h == 0.0 and g > 1.0
    idx, g, h = D.sha_offload_plan([1 << 30], 16)  # C1
    assert list(idx) == [0] and g == 0.0 and 0 < h < 5.0
    rng = np.random.default_rng(7)
    lens = np.exp(rng.uniform(np.log(4096), np.log(1 << 30), 1000)).astype(np.uint64)
    idx, g, h = D.sha_offload_plan(lens, 16)
    g0 = D.sha_offload_plan(lens, 0)[1]
    assert 0 < idx.size < lens.size and max(g, h) < 0.9 * g0
    order = np.argsort(-lens.astype(np.int64), kind="stable")
    assert np.array_equal(idx, order[:idx.size])  # the longest ones, longest first
    assert D.sha_offload_plan(lens, 0)[0].size == 0
    assert D.sha_offload_plan([], 16)[0].size == 0
    assert D.sha_offload_plan([0, 0, 0], 16)[0].size == 0
    with pytest.raises(Exception):
        D.sha_offload_plan(lens, -1)


def test_host_offload_plan_modes():
    """krk_host_offload_plan: blobs in host memory.  C2 (1,000 x 100 MiB) is bound by the
    host link, so with the whole-blob mode (hash + piece sums on the host, never uploaded)
    the host takes some blobs and the modelled makespan drops to the GPU's own chain time;
    a batch in HBM (KRK_OFFLOAD_DEVICE) keeps every equal blob on the GPU."""
    from kraken_amd import device as D
    c2 = [100 << 20] * 1000
    R = D.planner_rates()
    assert R["source"] == "nominal" and R["cus"] == 256  # no device here
    g0 = D.sha_offload_plan(c2, 0, mode=D.OFFLOAD_HOST_WHOLE)[1]
    assert abs(g0 - 1000 * (100 << 20) / (0.85 * R["h2d_bps"])) < 1e-6  # link-bound with no offload
    idx, g, h = D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_HOST_WHOLE)
    assert max(g, h) <= g0
    if idx.size:  # host cores with the SHA extensions: the link sheds the host's blobs
        assert max(g, h) < 0.97 * g0 and g >= (100 << 20) / R["sha_stream_bps"][0] - 1e-9
        assert sorted(idx.tolist()) == list(range(idx.size))  # equal lengths: stable order
    assert D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_DEVICE)[0].size == 0
    idx, g, h = D.sha_offload_plan([1 << 30], 4, mode=D.OFFLOAD_HOST_SHA)  # C1 from host memory
    assert list(idx) == [0] and g == 0.0 and h > 0
    # cache files (one read, SHA-256 + CRC a chunk on one thread): fewer blobs than the
    # whole-blob mode, whose two passes run on two threads
    idx_f, gf, hf = D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_HOST_FILES)
    assert max(gf, hf) <= g0 and idx_f.size <= D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_HOST_WHOLE)[0].size
    with pytest.raises(Exception):
        D.sha_offload_plan(c2, 4, mode=4)


def test_planner_moves_with_injected_rates():
    """the planner's rates are data (measured on the device at first
    use, krk_planner_rates_set to inject), not box constants.  Faster GPU streams keep a
    lone long blob on the GPU; a slower host link makes the host take more blobs of a
    host-resident C2 batch; more CUs move a 20,000-stream batch to a faster tier."""
    from kraken_amd import device as D
    nominal = D.planner_rates()
    try:
        fast_gpu = dict(nominal, sha_stream_bps=[4e9, 4e9, 4e9])
        D.set_planner_rates(fast_gpu)
        assert D.planner_rates()["source"] == "set"
        assert D.sha_offload_plan([1 << 30], 16)[0].size == 0  # GPU chain now beats the host thread
        D.set_planner_rates(dict(nominal, sha_stream_bps=[1e6, 1e6, 1e6]))
        assert list(D.sha_offload_plan([1 << 30], 16)[0]) == [0]
        c2 = [100 << 20] * 1000
        D.set_planner_rates(nominal)
        n_fast_link = D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_HOST_WHOLE)[0].size
        D.set_planner_rates(dict(nominal, h2d_bps=nominal["h2d_bps"] / 4))
        n_slow_link = D.sha_offload_plan(c2, 16, mode=D.OFFLOAD_HOST_WHOLE)[0].size
        assert n_slow_link > n_fast_link
        # 20,000 streams: one-lane tier on 256 CUs, two-lane tier on 512 CUs
        D.set_planner_rates(dict(nominal, sha_stream_bps=[60e6, 50e6, 10e6]))
        g256 = D.sha_offload_plan([1 << 20] * 20000, 0, cus=256)[1]
        g512 = D.sha_offload_plan([1 << 20] * 20000, 0, cus=512)[1]
        assert abs(g256 - 20000 * (1 << 20) / (128 * 256 * 10e6)) < 1e-9 or abs(g256 - (1 << 20) / 10e6) < 1e-9
        assert abs(g512 - (1 << 20) / 50e6) < 1e-9
        with pytest.raises(Exception):
            D.set_planner_rates(dict(nominal, d2h_bps=0.0))
    finally:
        D.set_planner_rates(None)
    assert D.planner_rates()["source"] == "nominal"


def test_library_loads_after_torch(tmp_path):
    """bench.py and the gloo tests import torch before the library; a PyTorch wheel brings
    its own (older) libamdhip64, so the library must not need a newer HIP symbol version at
    load time (no HIP 7.1-only call such as hipMemcpyBatchAsync is linked)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import torch; from kraken_amd import _capi; "
            "print(_capi.lib.krk_version().decode())" % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("kraken_amd"), r.stderr[-2000:]


def test_piece_sums_files_host_placement(tmp_path):
    """krk_piece_sums_files (+ _multi) on the host placement -- Generate over cache files
    (generator.go:41-58) read once in preads on the host pool, no device needed: every
    piece sum equals zlib over the file's bytes, and the reference's error texts hold."""
    import zlib
    from kraken_amd._capi import krk_file_blob
    rng = np.random.default_rng(31)
    lens = [0, 1, 63, 4096, (1 << 20) - 1, (1 << 20) + 1, (17 << 20) + 3, 40 << 20]
    datas = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    paths = []
    for i, d in enumerate(datas):
        p = tmp_path / f"f{i}"
        p.write_bytes(d)
        paths.append(str(p).encode())
    check(lib.krk_set_crc_placement(_capi.KRK_PLACE_HOST))
    try:
        for P in (1, 4097, 1 << 20, 4 << 20):
            if P == 1:
                use = [i for i, L in enumerate(lens) if L <= 4096]
            else:
                use = list(range(len(lens)))
            arr = (krk_file_blob * len(use))()
            off = 0
            for k, i in enumerate(use):
                arr[k] = krk_file_blob(paths[i], lens[i], P, off)
                off += int(lib.krk_num_pieces(lens[i], P))
            for fn in (lib.krk_piece_sums_files, lib.krk_piece_sums_files_multi):
                sums = np.zeros(max(off, 1), dtype=np.uint32)
                check(fn(arr, len(use), sums.ctypes.data_as(C.POINTER(C.c_uint32))))
                for k, i in enumerate(use):
                    d = datas[i]
                    want = [zlib.crc32(d[a:a + P]) for a in range(0, len(d), P)]
                    got = sums[arr[k].sums_offset:arr[k].sums_offset + len(want)]
                    assert list(got) == want, (P, i)
            g, h, _ = C.c_uint64(), C.c_uint64(), C.c_double()
            check(lib.krk_crc_host_split(C.byref(g), C.byref(h), C.byref(_)))
            assert g.value == 0 and h.value == sum(lens[i] for i in use)
        sums = np.zeros(64, dtype=np.uint32)
        bad = (krk_file_blob * 1)(krk_file_blob(paths[5], lens[5] + 10, 1 << 20, 0))
        assert lib.krk_piece_sums_files(bad, 1, sums.ctypes.data_as(C.POINTER(C.c_uint32))) == _capi.KRK_EIO
        assert lib.krk_last_error() == b"read blob: " + paths[5] + b": unexpected EOF"
        missing = str(tmp_path / "nope").encode()
        bad = (krk_file_blob * 1)(krk_file_blob(missing, 5, 1 << 20, 0))
        assert lib.krk_piece_sums_files(bad, 1, sums.ctypes.data_as(C.POINTER(C.c_uint32))) == _capi.KRK_EIO
        assert lib.krk_last_error() == b"open " + missing + b": No such file or directory"
        # an EMPTY missing file fails too (Generate opens the file before reading)
        bad = (krk_file_blob * 2)(krk_file_blob(paths[1], 1, 1 << 20, 0), krk_file_blob(missing, 0, 1 << 20, 1))
        assert lib.krk_piece_sums_files(bad, 2, sums.ctypes.data_as(C.POINTER(C.c_uint32))) == _capi.KRK_EIO
        assert lib.krk_last_error() == b"open " + missing + b": No such file or directory"
        bad = (krk_file_blob * 1)(krk_file_blob(missing, 0, 1 << 20, 0))
        assert lib.krk_piece_sums_files(bad, 1, sums.ctypes.data_as(C.POINTER(C.c_uint32))) == _capi.KRK_EIO
    finally:
        check(lib.krk_set_crc_placement(_capi.KRK_PLACE_AUTO))


def test_piece_sums_host_pageable_needs_no_device():
    """Pageable host buffers stay on host threads (krk_piece_sums_host / verify_pieces_host),
    so those calls run without a gfx950 device: sums equal zlib, verdicts follow them."""
    import zlib
    from kraken_amd import agentstorage
    from kraken_amd import device as D
    rng = np.random.default_rng(41)
    datas = [rng.integers(0, 256, L, dtype=np.uint8) for L in (0, 1, 4097, (3 << 20) + 5, 9 << 20)]
    for P in (1 << 20, 4097):
        for d, s in zip(datas, D.piece_sums_host(datas, P)):
            b = d.tobytes()
            assert [int(x) for x in s] == [zlib.crc32(b[k:k + P]) for k in range(0, len(b), P)]
    exp = np.array([zlib.crc32(d.tobytes()) for d in datas], dtype=np.uint32)
    exp[2] ^= 1
    assert list(agentstorage.verify_pieces(datas, exp)) == [True, True, False, True, True]


def test_host_hash_work_concurrent_callers_under_cpu_tokens():
    """Many concurrent host-placed callers (piece streams, crc32.Update, piece_sums_host)
    share the CPU tokens (at most the CPU budget hashing at once, host_pool.cpp): no caller
    deadlocks or starves, every result equals zlib."""
    import threading
    import zlib
    from kraken_amd import device as D
    rng = np.random.default_rng(61)
    blob = rng.integers(0, 256, (9 << 20) + 77, dtype=np.uint8)
    data = blob.tobytes()
    P = 2 << 20
    want = [zlib.crc32(data[i:i + P]) for i in range(0, len(data), P)]
    errors = []

    def stream_worker():
        try:
            for _ in range(3):
                s = C.c_void_p()
                check(lib.krk_piece_stream_begin_on(_capi.KRK_PLACE_HOST, P, C.byref(s)))
                try:
                    for a in range(0, len(data), 1 << 20):
                        chunk = data[a:a + (1 << 20)]
                        check(lib.krk_piece_stream_update(s, chunk, len(chunk)))
                    ns, ln = C.c_uint64(), C.c_uint64()
                    sums = (C.c_uint32 * len(want))()
                    check(lib.krk_piece_stream_end(s, sums, len(want), C.byref(ns), C.byref(ln)))
                    assert list(sums) == want
                finally:
                    lib.krk_piece_stream_free(s)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(e)

    def update_worker():
        try:
            for _ in range(3):
                out = C.c_uint32()
                check(lib.krk_crc32_update_on(_capi.KRK_PLACE_HOST, 0, data, len(data), C.byref(out)))
                assert out.value == zlib.crc32(data)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def batch_worker():
        try:
            for _ in range(2):
                got = D.piece_sums_host([blob, blob[:P + 1]], P)
                assert [int(x) for x in got[0]] == want
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = ([threading.Thread(target=stream_worker) for _ in range(24)] +
          [threading.Thread(target=update_worker) for _ in range(8)] +
          [threading.Thread(target=batch_worker) for _ in range(4)])
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a caller did not finish"
    assert not errors, errors[:3]


def test_public_header_is_the_bound_surface():
    """include/kraken_hip.h declares exactly what INTEGRATION.md's
    surface table binds (the Go callers' entry points and the operator calls); the
    benchmark / diagnostic hooks live in include/kraken_hip_internal.h only."""
    import os
    import re
    doc = open(os.path.join(os.path.dirname(_capi.HEADER_PATH), "..", "INTEGRATION.md")).read()
    a = doc.index("## The exported surface")
    b = doc.index("\n## ", a + 1)
    table = set(re.findall(r"`(krk_[a-z0-9_]+)`", doc[a:b]))
    pub, internal = set(_capi.public_symbols()), set(_capi.internal_symbols())
    assert pub == table, ("header only", sorted(pub - table), "table only", sorted(table - pub))
    assert not pub & internal
    hooks = {"krk_set_sha_plan", "krk_synth_fill_dev", "krk_synth_fill_chunks_dev", "krk_planner_rates_set",
             "krk_kernel_timeline", "krk_kernel_stats", "krk_set_timing", "krk_window_sched_new",
             "krk_window_sched_next", "krk_window_sched_free", "krk_windows_last_call", "krk_windows_last_direct",
             "krk_device_clock_mhz"}
    assert hooks <= internal, hooks - internal
    # every function the Go files in INTEGRATION.md call is public
    called = set(re.findall(r"\bC\.(krk_[a-z0-9_]+)\(", doc))
    assert called <= pub, called - pub


def _set_rates(stream, host_sha, h2d, cus=256):
    r = _capi.krk_planner_rates()
    for k, v in enumerate(stream):
        r.sha_stream_bps[k] = v
    r.d2h_bps = r.h2d_bps = h2d
    r.host_sha_bps, r.host_crc_bps, r.host_copy_bps = host_sha, 10e9, 10e9
    r.cus = cus
    check(lib.krk_planner_rates_set(C.byref(r)))


def test_digester_crossover_follows_injected_rates():
    """AUTO's Digester switch point comes from the planner rates: the
    fewest live GPU digesters whose aggregate (streams x per-stream rate x 0.93, capped by
    what the engine's zero-copy reads carry, 0.58 x the pinned H2D rate) beats the CPU budget
    x one thread's SHA-NI rate; none when the host out-hashes that (the MI355X box, measured:
    bench --workload engine's sweep never has the GPU ahead of 16 SHA-NI threads)."""
    import math
    cpus = _capi.host_cpu_budget()[0]
    n = C.c_int64()
    check(lib.krk_set_digester_host_streams(-1))
    try:
        for host_sha, stream in ((1e9, 57e6), (2e9, 57e6), (1e9, 30e6)):
            _set_rates([stream, 50e6, 35e6], host_sha, 200e9)  # a link wide enough not to cap
            check(lib.krk_digester_host_streams(C.byref(n)))
            want = math.floor(cpus * host_sha / (stream * 0.93)) + 1  # the first m that beats the host
            assert n.value == want - 1, (host_sha, stream, n.value, want)
        # a host that out-hashes what the engine carries over the link (0.58 x H2D): every AUTO
        # digester stays on the host (the MI355X box: 16 x 2.1 GB/s against 0.58 x 56.6)
        _set_rates([57e6, 50e6, 35e6], 2e9, cpus * 2e9 / 0.58 * 0.99)
        check(lib.krk_digester_host_streams(C.byref(n)))
        assert n.value >= (1 << 62)
        # an operator's pin wins over the rates
        check(lib.krk_set_digester_host_streams(123))
        check(lib.krk_digester_host_streams(C.byref(n)))
        assert n.value == 123
    finally:
        check(lib.krk_set_digester_host_streams(-1))
        check(lib.krk_planner_rates_set(None))


def _replay_tails(lens, idx, start, threads, r, h):
    """The plan's own schedule replayed: host threads take the chains in the plan's order
    (ascending GPU prefix), each when it is free AND the GPU has reached the prefix (start /
    r); the batch ends when the last host tail and the last GPU-only chain end."""
    import heapq
    free = [0.0] * threads
    end = 0.0
    for i, y in zip(idx, start):
        t = max(heapq.heappop(free), y / r)
        done = t + (lens[i] - y) / h
        heapq.heappush(free, done)
        end = max(end, done)
    on_gpu = set(range(len(lens))) - set(int(i) for i in idx)
    return max([end] + [lens[i] / r for i in on_gpu])


def test_sha_tail_plan_follows_rates():
    """Tail handoff of the host offload (offload.cpp tail_plan): every chain starts on the GPU
    and host threads finish the tails of the longest from the GPU's midstate.  C2's shape on
    16 threads at the box's rates (58.5 MB/s a GPU stream, 2.1 GB/s a SHA-NI thread as the
    planner reports it -- derated 15 %; a tail thread is priced at 0.98 of the rate measured,
    2.42 GB/s): the batch ends ~1.43 s instead of 1.79 (measured 1.429); one long chain (C1)
    goes to the host whole; prefixes are
    64-byte multiples below each chain's length, listed in ascending order; the plan's replay
    meets its own end; no host threads, no plan."""
    from kraken_amd import device as Dv
    try:
        _set_rates([58.5e6, 51.7e6, 34.9e6], 2.1e9, 55.9e9)
        L = [104857600] * 1000
        idx, start, end_s, gpu_s = Dv.sha_tail_plan(L, 16)
        assert len(idx) == 1000 and len(set(idx.tolist())) == 1000
        assert 1.38 < end_s < 1.47 and abs(gpu_s - 104857600 / 58.5e6) < 1e-6, (end_s, gpu_s)
        assert (start % 64 == 0).all() and (start < 104857600).all() and (np.diff(start.astype(np.int64)) >= 0).all()
        assert (start[:16] == 0).all() and start[-1] > 0  # the first takeovers are whole blobs
        h = 2.1e9 * 0.98 / 0.85  # a tail thread's rate (offload.cpp tail_plan)
        assert _replay_tails(L, idx, start, 16, 58.5e6, h) <= end_s * 1.001
        idx, start, end_s, gpu_s = Dv.sha_tail_plan([1 << 30] + [1 << 20] * 5, 16)
        assert 0 in idx.tolist() and start[idx.tolist().index(0)] == 0 and end_s < 0.6
        mixed = [(50 + 37 * k % 200) << 20 for k in range(300)]
        idx, start, end_s, gpu_s = Dv.sha_tail_plan(mixed, 8)
        assert end_s < gpu_s and _replay_tails(mixed, idx, start, 8, 58.5e6, h) <= end_s * 1.001
        assert all(start[k] < mixed[i] for k, i in enumerate(idx))
        assert Dv.sha_tail_plan(L, 0)[0].size == 0
    finally:
        check(lib.krk_planner_rates_set(None))


def test_window_sched_drop_and_chunk_cap():
    """The tail handoff's schedule hooks (no device): krk_window_sched_drop takes a live blob
    out (its offset = the bytes the windows gave it; its place goes to the next waiting
    blob) or a waiting one (offset 0, never admitted); krk_window_sched_set_chunk_cap bounds
    every later chunk.  Every other blob still gets every byte once, in order."""
    lens = np.array([9000, 7000, 5000, 3000, 1000], dtype=np.uint64)
    h = C.c_void_p()
    check(lib.krk_window_sched_new(lens.ctypes.data_as(C.POINTER(C.c_uint64)), 5, 4096, 2, C.byref(h)))
    b, o, t = np.zeros(8, np.uint32), np.zeros(8, np.uint64), np.zeros(8, np.uint64)
    k = C.c_uint64()

    def nxt():
        check(lib.krk_window_sched_next(h, b.ctypes.data_as(C.POINTER(C.c_uint32)), o.ctypes.data_as(
            C.POINTER(C.c_uint64)), t.ctypes.data_as(C.POINTER(C.c_uint64)), 8, C.byref(k)))
        return [(int(b[j]), int(o[j]), int(t[j])) for j in range(k.value)]

    try:
        w0 = nxt()
        assert [x[0] for x in w0] == [0, 1] and all(x[2] == 2048 for x in w0)  # longest first, 4096 / 2 live
        off = C.c_uint64()
        check(lib.krk_window_sched_drop(h, 0, C.byref(off)))
        assert off.value == 2048
        check(lib.krk_window_sched_drop(h, 3, C.byref(off)))  # still waiting
        assert off.value == 0
        with pytest.raises(RuntimeError, match="neither live nor waiting"):
            check(lib.krk_window_sched_drop(h, 3, C.byref(off)))
        check(lib.krk_window_sched_set_chunk_cap(h, 640))
        pos = {1: 2048, 2: 0, 4: 0}
        seen = set()
        while True:
            w = nxt()
            if not w:
                break
            for blob, offs, take in w:
                assert blob in pos and offs == pos[blob] and take <= 640, (blob, offs, take)
                pos[blob] += take
                seen.add(blob)
        assert pos == {1: 7000, 2: 5000, 4: 1000} and seen == {1, 2, 4}
    finally:
        lib.krk_window_sched_free(h)


def test_tail_handoff_model_accounts_every_byte():
    """windowed.simulate_tail_handoff (no device; the planner's rates injected): the policy
    the GPU run uses, on rank 0's LPT shard of an 8-GPU C3 scaled down 64x.  The threads'
    bytes plus the windows' bytes are the batch; the modelled end beats the GPU alone (the
    longest chain at the eight-lane rate) and is no earlier than the work allows (launches
    priced at 0 s at this scale)."""
    from kraken_amd.shard import lpt_shard
    from kraken_amd.windowed import c3_lengths, simulate_tail_handoff
    L = c3_lengths(20000, scale=64)
    lens = [L[i] for i in lpt_shard(L, 8)[0]]
    rates = {"sha_stream_bps": [58.5e6, 52.3e6, 35.2e6], "d2h_bps": 56e9, "h2d_bps": 56e9, "host_sha_bps": 2.1e9,
             "host_crc_bps": 17e9, "host_copy_bps": 30e9, "cus": 256, "source": 2}
    m = simulate_tail_handoff(lens, len(lens) * (64 << 10), len(lens), 15, rates, launch_s=0.0, max_chunk=64 << 10)
    gpu_only = max(lens) / 58.5e6
    assert m["end_s"] < 0.8 * gpu_only, (m, gpu_only)
    total = sum(lens)
    assert 0 < m["host_bytes"] < total
    # no faster than all of it on the host threads plus every GPU stream at once
    assert m["end_s"] >= total / (15 * m["thread_rate_Bps"] + len(lens) * 58.5e6)
    assert m["takeovers"] >= 15


def test_tail_ring_slot_held_until_its_crc_is_queued():
    """TailHandoffRun's ring (no device: a stand-in records every generation into a slot).  A
    thread may copy a piece down and free its slot before the loop has flushed that piece's
    CRC; the slot must not be regenerated until the CRC is queued and its event done -- the
    round-6 GPU failure was a 1 MiB-piece run whose ring wrapped inside one window wait and
    overwrote pieces whose CRCs had not run (wrong sums, right digests)."""
    import threading
    from kraken_amd import windowed as WN

    class Buf:
        def __init__(self, p):
            self.ptr = p

    class Lib:
        def __init__(self):
            self.done = {}

        def krk_event_query(self, ev, out):
            out._obj.value = int(self.done.get(ev.value, 0))
            return 0

        def krk_stream_sync(self, s):
            return 0

        def krk_memcpy_d2h_async(self, dst, src, n, s):
            return 0

        def krk_event_record(self, ev, s):
            return 0

    class FakeD:
        def __init__(self):
            self.lib = Lib()
            self.fills = []

        def check(self, rc):
            assert rc == 0

        def synth_fill_chunk_arrays(self, ids, ptr, off, n, stream=None):
            self.fills.extend(int(p) for p in ptr)

    D = FakeD()
    r = WN.TailHandoffRun.__new__(WN.TailHandoffRun)
    import time
    r.D, r.H, r.ring, r.piece, r._clock, r._gen_wait = D, 1, 2, 64, time.perf_counter, [0.0, 0.0]
    r.hbuf, r.slot_ev, r.copy_s = [[Buf(0x9000), Buf(0xA000)]], [[C.c_void_p(1), C.c_void_p(2)]], C.c_void_p()
    r.piece_s = C.c_void_p()
    r.ids = np.arange(4, dtype=np.uint64)
    r.gen_s = C.c_void_p()
    r.tbuf = [[Buf(0x1000), Buf(0x2000)]]
    r._cv = threading.Condition(threading.Lock())
    r._to_gen = [[(0, o, 64, 0) for o in range(0, 6 * 64, 64)]]
    r._ready, r._pending, r._tail_pieces = [[]], [], 0
    r._slot_used, r._slot_crc, r._next_slot = [[False, False]], [[None, None]], [0]
    assert len(r._service()) == 2  # both slots filled
    r._ready[0].clear()
    r._slot_used[0] = [False, False]  # the thread copied both down ...
    assert r._service() == [] and D.fills == [0x1000, 0x2000]  # ... but no CRC is queued yet
    take = r._pending[:]
    r._pending.clear()  # what _flush_crcs does, then _release with the event after it
    ev = C.c_void_p(77)
    r._release(take, ev)
    assert r._service() == []  # queued, not done
    D.lib.done[77] = 1
    assert len(r._service()) == 2 and D.fills[2:] == [0x1000, 0x2000]


def test_production_library_reads_only_the_operator_knobs():
    """the production library's environment is INTEGRATION.md's operator
    table, exactly -- every KRK_* name in its strings is in the table and every table entry is
    one it reads; the A/B switches of measurement sessions (knobs.hpp KRK_AB_ENV) are read by
    the diag build only.  Every library source reads its environment through knobs.hpp."""
    import glob
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    a = doc.index("## Operator knobs")
    b = doc.find("\n## ", a + 1)
    table = set()
    for line in doc[a:b if b > 0 else None].splitlines():
        if line.startswith("| `KRK_"):
            table |= set(re.findall(r"`(KRK_[A-Z0-9_]+)`", line.split("|")[1]))
    blob = open(_capi.LIB_PATH, "rb").read()
    names = set(re.findall(rb"KRK_[A-Z0-9_]+", blob))
    read = {n.decode() for n in names}
    assert read == table, ("read, not in the table", sorted(read - table), "table, not read", sorted(table - read))
    src = ""
    for p in glob.glob(os.path.join(root, "kraken_amd", "csrc", "*.[ch]*")):
        if not p.endswith("knobs.hpp"):
            src += open(p).read()
    bare = re.findall(r'getenv\("(KRK_[A-Z0-9_]+)"\)', src)
    assert not bare, f"KRK_* read outside knobs.hpp: {sorted(set(bare))}"
    op = set(re.findall(r'KRK_OP_ENV\("(KRK_[A-Z0-9_]+)"\)', src))
    ab = set(re.findall(r'KRK_AB_ENV\("(KRK_[A-Z0-9_]+)"\)', src))
    assert op == table and not op & ab, (sorted(op ^ table), sorted(op & ab))
