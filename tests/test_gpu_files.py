"""VERDICT r03 item 2 / SURVEY 8(f) row 3: upload and cache-fill verification fused with the
metainfo, from the CAS files themselves -- krk_metainfo_digest_files (+ _multi): each file is
read once (pread into the pinned windows, on the host pool) and that read feeds the
SHA-256 digest of uploader.verify / CAStore.WriteCacheFile (origin/blobserver/uploader.go:
74-94, lib/store/ca_store.go:99-135) AND the piece CRCs of Generator.Generate
(lib/metainfogen/generator.go:41-58), where the reference reads the file twice.

* Edge lengths x piece lengths against the oracle, with the host offload off and on (the
  planner's files then read, hashed and piece-summed in one pass on host threads) and with a
  small live cap (admission), plus the reference's error texts.
* The production window shape: 16,384 blobs of the C3 length law / 64 (1.6-16.8 MB) from
  files and from pinned host memory (krk_metainfo_digest_host) through the C++ window
  schedule -- 14,336 live streams (7/8 of the two-lane count) on the two-lane two-pair plan
  (KRK_SHA_PLAN_2LANE_2PAIR = 4, krk_kernel_timeline), late admission of the other 2,048 --
  every blob equal to the one-shot device path, the shortest, longest, a partial and a late
  blob equal to the oracle."""
import hashlib
import os
import resource

import numpy as np
import pytest

from kraken_amd import device as D
from kraken_amd._capi import KRK_EIO, KrakenError, check, krk_blob, lib
from kraken_amd.windowed import c3_lengths

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 63, 64, 65, 4095, 4096, 4097, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 3 * (1 << 20) + 5, 9_999_999]


def _write(tmp_path, name, data):
    p = str(tmp_path / name)
    with open(p, "wb") as f:
        f.write(memoryview(data))
    return p


@pytest.mark.parametrize("P", [1 << 20, 3, 4 << 20])
@pytest.mark.parametrize("mode", ["gpu", "offload", "cap3", "direct_aio", "direct_sync"])
def test_files_edge_lengths_match_oracle(gpu, orc, tmp_path, P, mode, monkeypatch):
    lens = EDGE if P != 3 else [0, 1, 2, 3, 4, 64, 65, 100_001]
    datas = [orc.synth(50 + i, L) for i, L in enumerate(lens)]
    paths = [_write(tmp_path, f"b{i}", d) for i, d in enumerate(datas)]
    if mode == "cap3":
        monkeypatch.setenv("KRK_LIVE_CAP", "3")
    if mode.startswith("direct"):  # O_DIRECT chunks: Linux AIO (the cold default) or preads
        monkeypatch.setenv("KRK_FILE_DIRECT", "1")
        monkeypatch.setenv("KRK_FILE_AIO", "1" if mode == "direct_aio" else "0")
    if mode == "offload":
        D.set_sha_host_offload(8)
        D.set_planner_rates(dict(D.planner_rates(), sha_stream_bps=[1e6, 1e6, 1e6]))  # the host takes files
    try:
        sums, dg = D.metainfo_digest_files(paths, lens, P)
        st = D.windows_last_call()
    finally:
        D.set_sha_host_offload(0)
        D.set_planner_rates(None)
    for i, d in enumerate(datas):
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), (i, lens[i])
        assert np.array_equal(sums[i], orc.calc_piece_sums(d, P)[1]), (i, lens[i])
    if mode == "offload":
        assert st["host_blobs"] > 0
    if mode == "cap3":
        assert st["max_live"] == 3 and st["windows"] >= len(lens) // 3
    if mode.startswith("direct"):
        assert st["direct_reads"], st


def test_direct_batch_live_files_match_the_link(gpu, orc, tmp_path, monkeypatch):
    """Round 6: a batch read O_DIRECT keeps at most as many files live as it takes the windows'
    streams to outrun the host link (h2d / the eight-lane per-stream rate, rounded up to 64,
    at least 256) -- larger disk requests for cold batches.  With injected rates (30 GB/s,
    60 MB/s a stream) that is 512 of 1,300 files; KRK_LIVE_CAP still wins; every output equals
    hashlib / the oracle."""
    rng = np.random.default_rng(77)
    lens = [int(x) for x in rng.integers(1, 40_000, 1300)]
    src = orc.synth(4242, max(lens))
    paths = [_write(tmp_path, f"d{i}", src[:L]) for i, L in enumerate(lens)]
    monkeypatch.setenv("KRK_FILE_DIRECT", "1")
    D.set_planner_rates(dict(D.planner_rates(), h2d_bps=30e9, sha_stream_bps=[60e6, 50e6, 35e6]))
    try:
        D.set_sha_host_offload(0)
        sums, dg = D.metainfo_digest_files(paths, lens, 1 << 14)
        st = D.windows_last_call()
        monkeypatch.setenv("KRK_LIVE_CAP", "700")
        sums2, dg2 = D.metainfo_digest_files(paths, lens, 1 << 14)
        st2 = D.windows_last_call()
    finally:
        D.set_planner_rates(None)
    assert st["direct_reads"] and st["max_live"] == 512, st
    assert st2["max_live"] == 700, st2
    for i in range(0, len(lens), 37):
        d = src[:lens[i]]
        assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(d, 1 << 14)[1]), i
    assert np.array_equal(dg2, dg) and all(np.array_equal(a, b) for a, b in zip(sums, sums2))


def test_files_cold_batch_stays_on_windows_under_auto(gpu, orc, tmp_path):
    """The batch's page-cache residency is sampled (mmap + mincore): files out of the cache are
    disk-bound wherever they are hashed, so AUTO sends none to host threads and reads them
    O_DIRECT through Linux AIO; the same files cached go to host threads (with rates that make
    the host worth it) and are read from the page cache.  Outputs equal the oracle both ways."""
    lens = [4 << 20] * 6 + [3 << 20, 1]
    datas = [orc.synth(700 + i, L) for i, L in enumerate(lens)]
    paths = [_write(tmp_path, f"c{i}", d) for i, d in enumerate(datas)]

    def drop():
        for p in paths:
            fd = os.open(p, os.O_RDONLY)
            try:
                os.fsync(fd)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            finally:
                os.close(fd)

    D.set_sha_host_offload(-1)
    D.set_planner_rates(dict(D.planner_rates(), sha_stream_bps=[1e6, 1e6, 1e6]))  # the host takes files
    try:
        drop()
        sums_c, dg_c = D.metainfo_digest_files(paths, lens, 1 << 20)
        cold = D.windows_last_call()
        for p in paths:  # into the page cache
            with open(p, "rb") as f:
                f.read()
        sums_w, dg_w = D.metainfo_digest_files(paths, lens, 1 << 20)
        warm = D.windows_last_call()
    finally:
        D.set_sha_host_offload(0)
        D.set_planner_rates(None)
    assert 0 <= cold["resident_sample"] < 0.5 and cold["host_blobs"] == 0, cold
    assert cold["direct_reads"], cold  # a cold batch reads O_DIRECT (Linux AIO)
    assert warm["resident_sample"] >= 0.5 and warm["host_blobs"] > 0 and not warm["direct_reads"], warm
    for i, d in enumerate(datas):
        want = hashlib.sha256(d.tobytes()).digest()
        assert bytes(dg_c[i]) == want and bytes(dg_w[i]) == want, i
        ref = orc.calc_piece_sums(d, 1 << 20)[1]
        assert np.array_equal(sums_c[i], ref) and np.array_equal(sums_w[i], ref), i


@pytest.mark.parametrize("mode", ["default", "direct_aio", "direct_sync"])
def test_files_errors_keep_reference_texts(gpu, orc, tmp_path, mode, monkeypatch):
    if mode != "default":  # the same texts from the O_DIRECT reads (Linux AIO or preads)
        monkeypatch.setenv("KRK_FILE_DIRECT", "1")
        monkeypatch.setenv("KRK_FILE_AIO", "1" if mode == "direct_aio" else "0")
    d = orc.synth(1, 1 << 20)
    p = _write(tmp_path, "short", d)
    with pytest.raises(KrakenError) as e:
        D.metainfo_digest_files([p], [(1 << 20) + 10], 1 << 20)  # stat said longer: EOF
    assert e.value.code == KRK_EIO and str(e.value).endswith(f"read blob: {p}: unexpected EOF")
    missing = str(tmp_path / "nope")
    with pytest.raises(KrakenError) as e:
        D.metainfo_digest_files([p, missing], [1 << 20, 5], 1 << 20)
    assert e.value.code == KRK_EIO and f"open {missing}: No such file or directory" in str(e.value)
    # an empty file is opened too -- missing, it fails like the reference
    with pytest.raises(KrakenError) as e:
        D.metainfo_digest_files([p, missing], [1 << 20, 0], 1 << 20)
    assert e.value.code == KRK_EIO and f"open {missing}: No such file or directory" in str(e.value)
    with pytest.raises(KrakenError, match="piece length must be positive"):
        D.metainfo_digest_files([p], [1 << 20], 0)
    # the library is usable after the failures
    sums, dg = D.metainfo_digest_files([p], [1 << 20], 1 << 20)
    assert bytes(dg[0]) == hashlib.sha256(d.tobytes()).digest()


def test_files_multi_equals_single(gpu, orc, tmp_path):
    lens = [int(x) for x in np.random.default_rng(5).integers(0, 6 << 20, 40)]
    datas = [orc.synth(900 + i, L) for i, L in enumerate(lens)]
    paths = [_write(tmp_path, f"m{i}", d) for i, d in enumerate(datas)]
    s1, d1 = D.metainfo_digest_files(paths, lens, 1 << 20)
    check(lib.krk_set_devices((C_int * 2)(0, 0), 2))
    try:
        s2, d2 = D.metainfo_digest_files(paths, lens, 1 << 20, multi=True)
    finally:
        check(lib.krk_set_devices(None, 0))
    assert np.array_equal(d1, d2) and all(np.array_equal(a, b) for a, b in zip(s1, s2))
    for i in (0, 17, 39):
        assert bytes(d1[i]) == hashlib.sha256(datas[i].tobytes()).digest()


from ctypes import c_int as C_int  # noqa: E402

_FD_CHILD = r"""
import hashlib, os, resource, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
from ctypes import c_int
# the process may hold few descriptors: the library's pool = soft limit - open now - 64
open_now = len(os.listdir("/proc/self/fd"))
soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
resource.setrlimit(resource.RLIMIT_NOFILE, (open_now + 64 + 48, hard))
from kraken_amd import device as D
from kraken_amd._capi import check, lib
D.set_device(0)
D.set_sha_host_offload(0)
tmp = sys.argv[2]
lens = [int(x) for x in np.random.default_rng(8).integers(0, 3 << 20, 300)]
paths = []
for i, L in enumerate(lens):
    p = os.path.join(tmp, "fd%d" % i)
    with open(p, "wb") as f:
        f.write(O.synth(4000 + i, L).tobytes())
    paths.append(p)
check(lib.krk_set_devices((c_int * 6)(0, 0, 0, 0, 0, 0), 6))  # six workers share the one budget
sums, dg = D.metainfo_digest_files(paths, lens, 1 << 20, multi=True)
for i in range(0, len(lens), 7):
    d = O.synth(4000 + i, lens[i])
    assert bytes(dg[i]) == hashlib.sha256(d.tobytes()).digest(), i
    assert np.array_equal(sums[i], O.calc_piece_sums(d, 1 << 20)[1]), i
print("fd ok", len(lens))
"""


def test_files_multi_share_one_fd_budget(gpu, tmp_path):
    """the *_multi workers (and concurrent callers) lease descriptors from ONE
    process-wide budget; with ~48 descriptors to spare, six workers over 300 files would each
    have taken the whole budget (EMFILE) before.  Fresh process: the budget is read once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _FD_CHILD, root, str(tmp_path)], capture_output=True, text=True,
                       timeout=300, cwd=root)
    assert r.returncode == 0 and "fd ok 300" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]

N, SCALE, P4 = 16384, 64, 4 << 20
SOURCES = 64  # blob i = a prefix of source i % 64 (1 GB of distinct bytes for 151 GB of blobs)


@pytest.fixture(scope="module")
def c3_law(gpu, orc, tmp_path_factory):
    lens = c3_lengths(N, scale=SCALE)
    top = max(lens)
    srcs = [orc.synth((3 << 40) + s, top) for s in range(SOURCES)]
    d = tmp_path_factory.mktemp("c3files")
    paths = []
    for s, x in enumerate(srcs):
        p = str(d / f"src{s}")
        with open(p, "wb") as f:
            f.write(memoryview(x))
        paths.append(p)
    # one-shot device reference: every blob a prefix of its source in HBM
    dev = D.DeviceBuffer(SOURCES * top)
    for s, x in enumerate(srcs):
        dev.from_host(x, s * top)
    n_p = [int(lib.krk_num_pieces(L, P4)) for L in lens]
    offs = np.zeros(N + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(n_p)
    arr = (krk_blob * N)()
    for i, L in enumerate(lens):
        arr[i] = krk_blob(dev.ptr + (i % SOURCES) * top, L, P4, int(offs[i]))
    sums_d = D.DeviceBuffer(int(offs[-1]) * 4)
    dg_d = D.DeviceBuffer(N * 32)
    check(lib.krk_metainfo_digest_dev(arr, N, sums_d.ptr, dg_d.ptr, None))
    D.synchronize()
    one = (sums_d.to_host(np.uint32, int(offs[-1])), dg_d.to_host(np.uint8, N * 32).reshape(N, 32))
    del dev, sums_d, dg_d
    return lens, srcs, paths, offs, one


def _expected_all(lens, srcs, orc):
    """Every blob's digest and piece sums without hashing 151 GB: blob i is a prefix of source
    i % 64, so one pass per source gives them all -- SHA-256 (hashlib = crypto/sha256) fed in
    order of length, a copy finalised at each blob's end; the full pieces' sums are the
    source's own (the oracle's calcPieceSums); a partial last piece's CRC (zlib = hash/crc32)
    carried along the blobs whose last piece is the same piece."""
    import zlib
    dg = np.zeros((N, 32), dtype=np.uint8)
    sums = [None] * N
    for s, x in enumerate(srcs):
        ids = sorted(range(s, N, SOURCES), key=lambda i: lens[i])
        full = orc.calc_piece_sums(x[:len(x) // P4 * P4], P4)[1]
        h, pos = hashlib.sha256(), 0
        crc, cpos, cpiece = 0, 0, -1
        for i in ids:
            L = lens[i]
            h.update(memoryview(x[pos:L]))
            pos = L
            dg[i] = np.frombuffer(h.copy().digest(), dtype=np.uint8)
            k = L // P4
            if L % P4:
                if k != cpiece:
                    crc, cpos, cpiece = 0, k * P4, k
                crc = zlib.crc32(memoryview(x[cpos:L]), crc)
                cpos = L
                sums[i] = np.concatenate([full[:k], np.array([crc], dtype=np.uint32)])
            else:
                sums[i] = np.asarray(full[:k], dtype=np.uint32)
    return sums, dg


def _check_against_one_shot_and_oracle(lens, srcs, offs, one, sums, dg, orc):
    s1, d1 = one
    assert np.array_equal(dg, d1)
    for i in range(N):
        assert np.array_equal(sums[i], s1[int(offs[i]):int(offs[i + 1])]), i
    # every one of the 16,384 blobs against the reference arithmetic
    want_sums, want_dg = _expected_all(lens, srcs, orc)
    bad = [i for i in range(N) if bytes(dg[i]) != bytes(want_dg[i])]
    assert not bad, bad[:8]
    bad = [i for i in range(N) if not np.array_equal(sums[i], want_sums[i])]
    assert not bad, bad[:8]
    L = np.asarray(lens)
    order = np.argsort(-L, kind="stable")
    late = int(order[14336])  # the first blob admitted after the initial 14,336
    partial = int(np.flatnonzero(L % P4)[0])
    for i in sorted({int(L.argmin()), int(L.argmax()), partial, late}):  # and a few the direct way
        data = srcs[i % SOURCES][:lens[i]]
        assert bytes(dg[i]) == hashlib.sha256(data.tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(data, P4)[1]), i


@pytest.mark.parametrize("source", ["files", "pinned"])
def test_c3_law_16384_blobs_production_windows(gpu, orc, c3_law, source):
    lens, srcs, paths, offs, one = c3_law
    cap = D.window_stream_cap()
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if source == "files" and soft < cap + 1024:  # what Go's runtime does at start-up (os package)
        resource.setrlimit(resource.RLIMIT_NOFILE, (min(hard, 1 << 20), hard))
    bufs = []
    try:
        with D.KernelTimer():
            if source == "files":
                sums, dg = D.metainfo_digest_files([paths[i % SOURCES] for i in range(N)], lens, P4)
            else:
                for x in srcs:  # the sources in pinned host memory (krk_host_alloc)
                    pa = D.PinnedArray((x.size,), np.uint8)
                    pa.a[:] = x
                    bufs.append(pa)
                datas = [bufs[i % SOURCES].a[:lens[i]] for i in range(N)]
                sums, dg = D.metainfo_digest_host(datas, P4)
            st = D.windows_last_call()
            tl = [(p, u) for p, u, _, _ in D.KernelTimer.timeline("sha256_multi")]
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
        bufs.clear()
    print(source, st, cap, tl[:3], len(tl))
    assert cap % 64 == 0 and cap == 14336 * D.device_cus() // 256  # 7/8 of the two-lane count
    want_live = cap if source == "pinned" or min(hard, 1 << 20) >= cap + 1024 else st["max_live"]
    assert st["max_live"] == want_live and st["host_blobs"] == 0
    if want_live == 14336:
        assert tl[0] == (4, 14336), tl[:3]  # KRK_SHA_PLAN_2LANE_2PAIR at the cap
    assert st["windows"] > 100  # late admission: live shrinks below the cap only at the end
    _check_against_one_shot_and_oracle(lens, srcs, offs, one, sums, dg, orc)


@pytest.mark.parametrize("mixed", [False, True])
def test_pinned_blobs_go_direct(gpu, orc, mixed):
    """krk_metainfo_digest_host over page-locked blobs (krk_host_alloc): windows of few chunks
    are DMA'd from the caller's memory straight into the device window (no staging copy:
    krk_windows_last_direct); one pageable blob in the batch stages every window.  Outputs
    equal the oracle either way."""
    lens = [0, 5, (64 << 20) + 1, (100 << 20) + 7, 3 << 20, (300 << 20) + 3]
    datas, bufs = [], []
    for i, L in enumerate(lens):
        x = orc.synth(7000 + i, L)
        if mixed and i == 2:
            datas.append(x)
            continue
        pa = D.PinnedArray((max(L, 1),), np.uint8)
        pa.a[:L] = x
        bufs.append(pa)
        datas.append(pa.a[:L])
    try:
        sums, dg = D.metainfo_digest_host(datas, P4)
        st = D.windows_last_call()
        for i, L in enumerate(lens):
            x = np.asarray(datas[i])
            assert bytes(dg[i]) == hashlib.sha256(x.tobytes()).digest(), i
            assert np.array_equal(sums[i], orc.calc_piece_sums(x, P4)[1]), i
    finally:
        bufs.clear()
    assert st["windows"] >= 2 and st["host_blobs"] == 0
    assert st["direct_windows"] == (0 if mixed else st["windows"]), st


def test_piece_sums_files_placements_agree(gpu, orc, tmp_path):
    """krk_piece_sums_files on each CRC placement (host preads + PCLMUL on the host pool, GPU
    windows + CRC kernel, and AUTO = the measured crossover) gives the oracle's sums; the
    split report names the side that ran."""
    lens = EDGE + [(40 << 20) + 3]
    datas = [orc.synth(4000 + i, L) for i, L in enumerate(lens)]
    paths = [_write(tmp_path, f"p{i}", d) for i, d in enumerate(datas)]
    got = {}
    try:
        for name, place in (("host", D.PLACE_HOST), ("gpu", D.PLACE_GPU), ("auto", D.PLACE_AUTO)):
            D.set_crc_placement(place)
            got[name] = D.piece_sums_files(paths, lens, 1 << 20)
            g, h, _ = D.crc_host_split()
            if name != "auto":
                assert (g > 0) == (name == "gpu") and g + h == sum(lens), (name, g, h)
    finally:
        D.set_crc_placement(D.PLACE_GPU)  # the suite's setting (conftest)
    sums, offs = got["host"]
    for name in ("gpu", "auto"):
        assert np.array_equal(got[name][0], sums), name
    for i, d in enumerate(datas):
        assert np.array_equal(sums[int(offs[i]):int(offs[i + 1])], orc.calc_piece_sums(d, 1 << 20)[1]), i


def test_sha256_host_window_schedule(gpu, orc):
    """krk_sha256_host runs the C++ window schedule (no CRC): 20,000 blobs -- more than the
    live cap -- from pageable memory, every digest equal to hashlib, at most the cap live,
    late admission over several windows; empty and one-byte blobs included."""
    import ctypes as C
    n = 20000
    rng = np.random.default_rng(2024)
    lens = [int(x) for x in rng.integers(0, 300_000, n)]
    lens[0], lens[1], lens[-1] = 0, 1, 1 << 20
    src = orc.synth(99, max(lens) + 4096)
    offs = [int(x) for x in rng.integers(0, 4096, n)]
    datas = [src[o:o + L] for o, L in zip(offs, lens)]
    ptrs = (C.c_void_p * n)(*[d.ctypes.data if d.size else None for d in datas])
    ln = np.asarray(lens, dtype=np.uint64)
    out = np.zeros((n, 32), dtype=np.uint8)
    check(lib.krk_sha256_host(ptrs, ln.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                              out.ctypes.data_as(C.POINTER(C.c_uint8))))
    st = D.windows_last_call()
    cap = D.window_stream_cap()
    assert st["max_live"] == cap and st["windows"] >= 2 and st["host_blobs"] == 0, st
    for i in range(n):
        assert bytes(out[i]) == hashlib.sha256(datas[i].tobytes()).digest(), (i, lens[i])


def test_concurrent_host_paths_under_cpu_tokens(gpu, orc, tmp_path):
    """Host paths that share the CPU tokens, at once from several threads: end-to-end batches
    with the host offload on (offload threads + pool copies), files on the host CRC
    placement (pool preads), host piece streams and crc32.Update calls.  No caller stalls;
    every result equals hashlib / zlib / the oracle."""
    import threading
    import zlib
    from ctypes import c_uint32, c_uint64, c_void_p, byref
    from kraken_amd import _capi
    rng = np.random.default_rng(404)
    blobs = [orc.synth(6000 + i, int(n)) for i, n in enumerate(rng.integers(1, 12 << 20, 24))]
    paths = [_write(tmp_path, f"t{i}", b) for i, b in enumerate(blobs)]
    lens = [int(b.size) for b in blobs]
    P = 1 << 20
    want_dg = [hashlib.sha256(b.tobytes()).digest() for b in blobs]
    errors = []

    def e2e():
        try:
            for _ in range(2):
                sums, dg = D.metainfo_digest_host(blobs, P)
                assert [bytes(x) for x in dg] == want_dg
                assert np.array_equal(sums[5], orc.calc_piece_sums(blobs[5], P)[1])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def files():
        try:
            for _ in range(2):
                sums, offs = D.piece_sums_files(paths, lens, P)
                for i in (0, 7, 23):
                    assert np.array_equal(sums[int(offs[i]):int(offs[i + 1])], orc.calc_piece_sums(blobs[i], P)[1])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def streams(i):
        try:
            data = blobs[i].tobytes()
            s = c_void_p()
            check(lib.krk_piece_stream_begin_on(_capi.KRK_PLACE_HOST, P, byref(s)))
            try:
                for a in range(0, len(data), 3 << 20):
                    check(lib.krk_piece_stream_update(s, data[a:a + (3 << 20)], len(data[a:a + (3 << 20)])))
                n, ln = c_uint64(), c_uint64()
                out = (c_uint32 * ((len(data) + P - 1) // P))()
                check(lib.krk_piece_stream_end(s, out, len(out), byref(n), byref(ln)))
                assert list(out) == [zlib.crc32(data[k:k + P]) for k in range(0, len(data), P)]
            finally:
                lib.krk_piece_stream_free(s)
            o = c_uint32()
            check(lib.krk_crc32_update_on(_capi.KRK_PLACE_HOST, 0, data, len(data), byref(o)))
            assert o.value == zlib.crc32(data)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    D.set_sha_host_offload(-1)
    D.set_crc_placement(D.PLACE_HOST)
    try:
        th = ([threading.Thread(target=e2e) for _ in range(2)] + [threading.Thread(target=files) for _ in range(2)] +
              [threading.Thread(target=streams, args=(i,)) for i in range(12)])
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in th), "a caller did not finish"
    finally:
        D.set_sha_host_offload(0)
        D.set_crc_placement(D.PLACE_GPU)
    assert not errors, errors[:3]


def test_tiny_window_many_live_blobs(gpu, orc, monkeypatch):
    """with a 1 MiB window (KRK_WINDOW_MB=1) and 30,000 live blobs
    (KRK_LIVE_CAP), every live blob still advances by the schedule's 64-byte minimum chunk,
    1.9 MB a window: the staging lease must hold that, not W + 16 x live."""
    monkeypatch.setenv("KRK_WINDOW_MB", "1")
    monkeypatch.setenv("KRK_LIVE_CAP", "30000")
    lens = [100 + (i % 37) for i in range(30000)]
    datas = [orc.synth(7000 + i, L) for i, L in enumerate(lens)]
    D.set_sha_host_offload(0)
    sums, dg = D.metainfo_digest_host(datas, 64)
    st = D.windows_last_call()
    assert st["max_live"] == 30000 and st["windows"] >= 2, st
    for i in range(0, len(lens), 997):
        assert bytes(dg[i]) == hashlib.sha256(datas[i].tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(datas[i], 64)[1]), i
