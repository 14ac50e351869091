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
    n = C.c_int(-1)
    check(lib.krk_device_count(C.byref(n)))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    assert lib.krk_digester_new(C.byref(h)) == KRK_ENODEV
    assert lib.krk_piece_stream_begin(4, C.byref(h)) == KRK_ENODEV
    out = C.c_uint32()
    assert lib.krk_crc32_update(0, b"abc", 3, C.byref(out)) == KRK_ENODEV
    assert b"no HIP device" in lib.krk_last_error()


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
    """The SHA-NI compressor (when this CPU has it) and the portable one agree."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "ih.py"
    f.write_text(_IH_SCRIPT)
    runs = [subprocess.run([sys.executable, str(f), root], capture_output=True, text=True,
                           env={**os.environ, "KRK_SHA1_PORTABLE": v}) for v in ("0", "1")]
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
