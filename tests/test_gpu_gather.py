"""host-resident batches with ONE host-DRAM read a byte -- the caller's
pages made page-locked (pinned blobs as they are; pageable ones registered with
hipHostRegister for the call) and every window gathered into HBM by one launch of the
gather kernel (gather.hip), which reads them over PCIe.  Bit-exactness against the oracle
for unaligned starts (every residue mod 16), lengths around the 16-byte word and the page,
blobs that share pages (views of one buffer), a blob that ends at the last byte before an
inaccessible page (no load may leave the blob's pages), read-only memory (registration may
be refused: the windows stage instead), and pinned blobs in windows too wide for one DMA a
chunk.  Forced modes run in fresh processes (KRK_HOST_GATHER is read once)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from kraken_amd import device as D

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import ctypes as C, hashlib, json, mmap, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from kraken_amd import device as D
from oracle import oracle as O
D.set_device(0)
D.set_sha_host_offload(0)
P = int(sys.argv[2])
out = {"ok": True, "cases": {}}

def check(name, datas):
    sums, dg = D.metainfo_digest_host(datas, P)
    st = D.windows_last_call()
    ok = True
    for i, d in enumerate(datas):
        b = d.tobytes()
        ok = ok and bytes(dg[i]) == hashlib.sha256(b).digest()
        ok = ok and np.array_equal(sums[i], O.calc_piece_sums(np.frombuffer(b, np.uint8), P)[1])
    ptrs = (C.c_void_p * len(datas))(*[d.ctypes.data if d.size else None for d in datas])
    lens = np.array([d.size for d in datas], np.uint64)
    dg2 = np.zeros((len(datas), 32), np.uint8)
    D.check(D.lib.krk_sha256_host(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), len(datas),
                                  dg2.ctypes.data_as(C.POINTER(C.c_uint8))))
    ok = ok and np.array_equal(dg, dg2)
    out["cases"][name] = {"ok": bool(ok), "windows": st["windows"], "gather_windows": st["gather_windows"],
                          "registered_bytes": st["registered_bytes"]}
    out["ok"] = out["ok"] and bool(ok)

rng = np.random.default_rng(11)
edge = [0, 1, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 8191, 65535, 65536, 65537, (1 << 20) + 7, 3_000_001]
# 1. separately allocated blobs at every start residue mod 16
datas = []
for k, L in enumerate(edge * 2):
    r = k % 16
    base = rng.integers(0, 256, L + r + 16, dtype=np.uint8)
    datas.append(base[r:r + L])
check("residues", datas)
# 2. views of ONE buffer: neighbouring blobs share pages (the registry merges their ranges)
big = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
views, o = [], 3
for k in range(40):
    L = int(rng.integers(0, 600_000))
    views.append(big[o:o + L])
    o += L + int(rng.integers(0, 40))
check("shared_pages", views)
# 3. blobs ending at the last byte before a PROT_NONE page, odd starts and odd lengths: a load
#    past the blob's pages would fault
PAGE, NP = 4096, 260
m = mmap.mmap(-1, (NP + 1) * PAGE)
full = np.frombuffer(m, dtype=np.uint8)
full[:NP * PAGE] = rng.integers(0, 256, NP * PAGE, dtype=np.uint8)
libc = C.CDLL(None)
libc.mprotect.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
assert libc.mprotect(full.ctypes.data + NP * PAGE, PAGE, 0) == 0
end = NP * PAGE
tail = [full[end - L:end] for L in (PAGE * 2 + 7, PAGE + 1, 23, 9, (1 << 20) + 5)]
check("page_end", tail)
# 4. read-only memory (np.frombuffer of bytes): registration may be refused -> staged
ro = [np.frombuffer(rng.bytes(L), dtype=np.uint8) for L in (1 << 20, 3_000_017, 5)]
check("read_only", ro)
print(json.dumps(out))
"""


@pytest.mark.parametrize("mode", ["1", "0"])
def test_gather_edges_bit_exact(gpu, mode):
    env = dict(os.environ, KRK_HOST_GATHER=mode)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(1 << 20)], capture_output=True, text=True,
                       timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["ok"], res
    if mode == "1":
        for name in ("residues", "shared_pages", "page_end"):
            assert res["cases"][name]["gather_windows"] == res["cases"][name]["windows"] > 0, (name, res)
    else:
        assert all(c["gather_windows"] == 0 for c in res["cases"].values()), res


def test_gather_default_large_pageable_and_pinned_wide(gpu, orc):
    """The defaults (KRK_HOST_GATHER unset): a 320 MiB pageable batch stages (registering
    4 KiB pages measured slower than the staging copy); 200 pinned blobs
    (krk_host_alloc) in windows of more than 64 chunks are gathered without registration;
    both bit-exact."""
    D.set_sha_host_offload(0)
    lens = [(1 << 20) + 13 * i for i in range(320)]
    datas = [orc.synth(3000 + i, L) for i, L in enumerate(lens)]
    sums, dg = D.metainfo_digest_host(datas, 4 << 20)
    st = D.windows_last_call()
    assert st["gather_windows"] == 0 and st["registered_bytes"] == 0 and st["windows"] > 0, st
    for i in range(0, len(lens), 37):
        assert bytes(dg[i]) == hashlib.sha256(datas[i].tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(datas[i], 4 << 20)[1]), i
    pins = []
    for i in range(200):
        pa = D.PinnedArray((100_003 + i,), np.uint8)
        pa.a[:] = orc.synth(5000 + i, pa.a.size)
        pins.append(pa)
    pd = [p.a for p in pins]
    sums, dg = D.metainfo_digest_host(pd, 1 << 16)
    st = D.windows_last_call()
    assert st["gather_windows"] >= 1 and st["registered_bytes"] == 0, st
    for i in range(0, 200, 19):
        assert bytes(dg[i]) == hashlib.sha256(pd[i].tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(pd[i], 1 << 16)[1]), i
    # the CRC-only host batch over the same pinned blobs: wide windows gathered too
    got = D.piece_sums_host(pd, 1 << 16)
    for i in range(0, 200, 23):
        assert np.array_equal(got[i], orc.calc_piece_sums(pd[i], 1 << 16)[1]), i


def test_copyout_shares_page_with_registered_blob(gpu, orc):
    """under the gather of pageable blobs (KRK_HOST_GATHER=1), a tiny
    blob and the call's output arrays carved from ONE 4 KiB page of one page-aligned
    buffer, for both host-buffer entry points (krk_metainfo_digest_host, krk_sha256_host).
    The registry rounds the blob out to that whole page, so the outputs sit in a page the
    call registered: every call must release its registrations before the copy-out
    (windows.cpp release_caller_pages), report none live at it, and be bit-exact."""
    import ctypes as C
    import mmap

    PAGE = 4096
    m = mmap.mmap(-1, 64 * PAGE)
    buf = np.frombuffer(m, dtype=np.uint8)
    assert buf.ctypes.data % PAGE == 0
    P = 1 << 12
    lens = [200, 3 * PAGE + 17, 20 * PAGE + 5, 1, 0, 9 * PAGE]
    blobs, o = [], PAGE  # page 0 holds the tiny blob and the outputs; the rest follow it
    for L in lens[1:]:
        blobs.append(buf[o:o + L])
        o += L + 3
    tiny = buf[64:64 + lens[0]]
    datas = [tiny] + blobs
    for k, d in enumerate(datas):
        d[:] = orc.synth(7000 + k, d.size)
    n = len(datas)
    counts = [int(D.lib.krk_num_pieces(int(d.size), P)) for d in datas]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(counts)
    dg_off, sums_off = 1024, 2048  # both inside page 0, after the tiny blob
    assert dg_off >= 64 + lens[0] and sums_off >= dg_off + 32 * n and sums_off + 4 * int(offs[-1]) <= PAGE
    dg = buf[dg_off:dg_off + 32 * n]
    sums = buf[sums_off:sums_off + 4 * int(offs[-1])].view(np.uint32)
    arr = (D.krk_blob * n)()
    for i, d in enumerate(datas):
        arr[i] = D.krk_blob(d.ctypes.data if d.size else None, int(d.size), P, int(offs[i]))
    D.set_sha_host_offload(0)
    D.set_host_gather(1)
    try:
        for rep in range(3):
            dg[:] = 0
            sums[:] = 0
            D.check(D.lib.krk_metainfo_digest_host(arr, n, sums.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                   dg.ctypes.data_as(C.POINTER(C.c_uint8))))
            st = D.windows_last_call()
            assert st["gather_windows"] == st["windows"] > 0 and st["registered_bytes"] > 0, st
            assert st["live_registered_at_copyout"] == 0, st
            for i, d in enumerate(datas):
                b = d.tobytes()
                assert bytes(dg[32 * i:32 * i + 32]) == hashlib.sha256(b).digest(), (rep, i)
                ref = orc.calc_piece_sums(np.frombuffer(b, np.uint8), P)[1]
                assert np.array_equal(sums[int(offs[i]):int(offs[i + 1])], ref), (rep, i)
            # the Digester batch: its digests into the same page as the tiny blob
            ptrs = (C.c_void_p * n)(*[d.ctypes.data if d.size else None for d in datas])
            L = np.array([d.size for d in datas], np.uint64)
            dg[:] = 0
            D.check(D.lib.krk_sha256_host(ptrs, L.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                          dg.ctypes.data_as(C.POINTER(C.c_uint8))))
            st = D.windows_last_call()
            assert st["gather_windows"] == st["windows"] > 0 and st["live_registered_at_copyout"] == 0, st
            for i, d in enumerate(datas):
                assert bytes(dg[32 * i:32 * i + 32]) == hashlib.sha256(d.tobytes()).digest(), (rep, i)
    finally:
        D.set_host_gather(-1)
        D.set_sha_host_offload(-1)


def test_gather_mixed_pinned_mappings(gpu, orc):
    """a batch mixing krk_host_alloc blobs with page-locked memory the caller
    registered itself (hipHostRegister) -- the gather reads every blob at its host address,
    so every blob's mapping is checked before a window is gathered (staging.hpp MappedAtHost),
    not the first blob's alone.  Windows of more than 64 chunks (the gather's domain);
    bit-exact whichever path each window takes."""
    import ctypes as C
    import mmap

    hip = C.CDLL(D.lib._name)  # the HIP runtime the library itself links (not another copy in the process)
    hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    hip.hipHostUnregister.argtypes = [C.c_void_p]
    m = mmap.mmap(-1, 32 << 20)
    buf = np.frombuffer(m, dtype=np.uint8)
    assert hip.hipHostRegister(buf.ctypes.data, buf.size, 0) == 0
    try:
        pins, datas, o = [], [], 0
        for i in range(160):
            L = 70_001 + 37 * i
            if i % 2:
                pa = D.PinnedArray((L,), np.uint8)
                pa.a[:] = orc.synth(9000 + i, L)
                pins.append(pa)
                datas.append(pa.a)
            else:
                v = buf[o + (i % 13):o + (i % 13) + L]
                v[:] = orc.synth(9000 + i, L)
                datas.append(v)
                o += L + 64
        D.set_sha_host_offload(0)
        sums, dg = D.metainfo_digest_host(datas, 1 << 16)
        st = D.windows_last_call()
        assert st["windows"] > 0 and st["registered_bytes"] == 0, st
        for i in range(0, len(datas), 7):
            assert bytes(dg[i]) == hashlib.sha256(datas[i].tobytes()).digest(), i
            assert np.array_equal(sums[i], orc.calc_piece_sums(datas[i], 1 << 16)[1]), i
        got = D.piece_sums_host(datas, 1 << 16)
        for i in range(0, len(datas), 9):
            assert np.array_equal(got[i], orc.calc_piece_sums(datas[i], 1 << 16)[1]), i
        print("mixed mappings:", st)
    finally:
        D.set_sha_host_offload(-1)
        hip.hipHostUnregister(buf.ctypes.data)
