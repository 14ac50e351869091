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
