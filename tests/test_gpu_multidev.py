"""One process, several devices (origin/cmd/cmd.go:164 is one process):
the *_multi entry points LPT-split a batch over the process's device set and gather
every blob's results into the caller's arrays.  On the one-GPU test box the set lists
device 0 twice: two host workers share the GPU, which exercises the split, the
per-worker re-based sums and the gather exactly as eight devices would."""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

from kraken_amd import device as D
from kraken_amd._capi import KRK_ENODEV, check, krk_blob, krk_file_blob, lib

pytestmark = pytest.mark.gpu


@pytest.fixture
def two_workers(gpu):
    D.set_devices([0, 0])
    assert D.get_devices() == [0, 0]
    yield
    D.set_devices([])
    assert D.get_devices() == [0]


def _blobs(seed, n=23):
    rng = np.random.default_rng(seed)
    lens = [int(x) for x in rng.integers(0, 3 << 20, n)] + [0, 1, 4096, 5 << 20]
    return [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]


def test_metainfo_digest_host_multi(two_workers, orc):
    datas = _blobs(1)
    pls = [1 << 20 if i % 2 else 65536 for i in range(len(datas))]
    sums, dg = D.metainfo_digest_host(datas, pls, multi=True)
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(d, pls[i])[1]), i


def test_piece_sums_and_sha_host_multi(two_workers, orc):
    datas = _blobs(2)
    P = 1 << 18
    n = len(datas)
    counts = [int(lib.krk_num_pieces(d.size, P)) for d in datas]
    offs = np.concatenate(([0], np.cumsum(counts)))
    arr = (krk_blob * n)(*[krk_blob(d.ctypes.data if d.size else None, d.size, P, int(offs[i]))
                           for i, d in enumerate(datas)])
    sums = np.zeros(int(offs[-1]), dtype=np.uint32)
    check(lib.krk_piece_sums_host_multi(arr, n, sums.ctypes.data_as(C.POINTER(C.c_uint32))))
    for i, d in enumerate(datas):
        assert np.array_equal(sums[offs[i]:offs[i + 1]], orc.calc_piece_sums(d, P)[1]), i
    ptrs = (C.c_void_p * n)(*[d.ctypes.data if d.size else None for d in datas])
    lens = np.array([d.size for d in datas], dtype=np.uint64)
    dg = np.zeros((n, 32), dtype=np.uint8)
    check(lib.krk_sha256_host_multi(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                    dg.ctypes.data_as(C.POINTER(C.c_uint8))))
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i


def test_piece_sums_files_multi(two_workers, orc, tmp_path):
    datas = _blobs(3, n=9)
    P = 1 << 20
    paths = []
    for i, d in enumerate(datas):
        p = tmp_path / f"blob{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p).encode())
    counts = [int(lib.krk_num_pieces(d.size, P)) for d in datas]
    offs = np.concatenate(([0], np.cumsum(counts)))
    arr = (krk_file_blob * len(datas))(*[krk_file_blob(paths[i], d.size, P, int(offs[i]))
                                          for i, d in enumerate(datas)])
    sums = np.zeros(int(offs[-1]), dtype=np.uint32)
    check(lib.krk_piece_sums_files_multi(arr, len(datas), sums.ctypes.data_as(C.POINTER(C.c_uint32))))
    for i, d in enumerate(datas):
        assert np.array_equal(sums[offs[i]:offs[i + 1]], orc.calc_piece_sums(d, P)[1]), i
    # a missing file fails the whole call with the reference's error text
    arr[0] = krk_file_blob(str(tmp_path / "missing").encode(), 10, P, 0)
    assert lib.krk_piece_sums_files_multi(arr, len(datas), sums.ctypes.data_as(C.POINTER(C.c_uint32))) != 0
    assert b"missing" in lib.krk_last_error()


def test_device_set_rejects_absent_device(gpu):
    bad = (C.c_int * 1)(4096)
    assert lib.krk_set_devices(bad, 1) == KRK_ENODEV
    assert D.get_devices() == [0]


def test_metainfo_digest_host_multi_with_offload(two_workers, orc):
    """The *_multi split with the SHA-256 host offload on: each worker's batch hands its
    longest blobs to host threads (the two workers share one device context, so their
    offload phases take turns on its thread pool); results equal hashlib / the oracle."""
    rng = np.random.default_rng(9)
    datas = [rng.integers(0, 256, L, dtype=np.uint8) for L in
             [(20 << 20) + 1, 12 << 20, 9 << 20] + [int(x) for x in rng.integers(0, 1 << 20, 30)]]
    try:
        D.set_sha_host_offload(4)
        sums, dg = D.metainfo_digest_host(datas, 1 << 20, multi=True)
    finally:
        D.set_sha_host_offload(0)
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(d, 1 << 20)[1]), i


def test_eight_workers_share_the_host(gpu, orc):
    """the device set at 8 entries (device 0 eight times here) -- the
    LPT split, 8 concurrent workers each with its share of the host threads (their copy
    threads no longer 8 x 16), the gather -- with every blob equal to the oracle."""
    D.set_devices([0] * 8)
    try:
        assert D.get_devices() == [0] * 8
        datas = _blobs(8, n=61)
        P = 1 << 20
        sums, dg = D.metainfo_digest_host(datas, [P] * len(datas), multi=True)
        for i, d in enumerate(datas):
            assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i
            assert np.array_equal(sums[i], orc.calc_piece_sums(d, P)[1]), i
    finally:
        D.set_devices([])
