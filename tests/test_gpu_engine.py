"""The submission engine behind the streaming entry points (engine.cpp): concurrent
Digesters / piece streams / crc32.Update calls coalesced into multi-stream launches,
pooled pinned staging, per-owner ordering; the host crossovers.  Reference callers:
origin/blobserver/uploader.go:75 and lib/store/ca_store.go:119 (a Digester per upload /
cache fill, many goroutines), lib/torrent/storage/agentstorage/torrent.go:182 (a
PieceHash per received piece).  Every result is checked against hashlib / zlib."""
import ctypes as C
import hashlib
import io
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from kraken_amd import core
from kraken_amd._capi import KRK_PLACE_AUTO, KRK_PLACE_GPU, KRK_PLACE_HOST, check, lib

pytestmark = pytest.mark.gpu

SLOT = 512 << 10  # the engine's default slot (KRK_SLOT_KB)


def _stats():
    v = [C.c_uint64() for _ in range(5)]
    check(lib.krk_engine_stats(*[C.byref(x) for x in v]))
    return [x.value for x in v]


def _feed(d, data: bytes, rng):
    i = 0
    while i < len(data):
        k = int(rng.integers(1, 1 << int(rng.integers(1, 21))))
        d._write(data[i:i + k])
        i += k


@pytest.mark.parametrize("placement", [KRK_PLACE_GPU, KRK_PLACE_HOST])
def test_digester_semantics(gpu, placement):
    """core/digester_test.go: the sha256("test") KAT, the empty digest (DigestEmptyTar),
    Digest() without reset (writing continues), lengths around the engine's slot size,
    random write sizes."""
    d = core.Digester(placement)
    assert d.placement() == placement
    assert d.Digest().String() == core.DigestEmptyTar
    d._write(b"test")
    assert d.Digest().Hex() == "9f86d081884c7d659a2feaa0c55ad015a3bf4f1b2b0b822cd15d6c15b0f00a08"
    assert d.Digest().Hex() == hashlib.sha256(b"test").hexdigest()  # no reset, idempotent
    d._write(b"more")
    assert d.Digest().Hex() == hashlib.sha256(b"testmore").hexdigest()
    rng = np.random.default_rng(placement)
    for n in [63, 64, 65, SLOT - 1, SLOT, SLOT + 1, 2 * SLOT + 55, 5 * SLOT + 17]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        d = core.Digester(placement)
        _feed(d, data, rng)
        h = hashlib.sha256(data[: n // 2])
        h.update(data[n // 2:])
        assert d.Digest().Hex() == h.hexdigest(), (placement, n)
        d._write(b"x")
        assert d.Digest().Hex() == hashlib.sha256(data + b"x").hexdigest(), (placement, n)
    assert core.Digester(placement).FromReader(io.BytesIO(b"abc")).Hex() == hashlib.sha256(b"abc").hexdigest()


def test_auto_placement_crossover(gpu):
    """KRK_PLACE_AUTO: host while at most N digesters are live in the process, GPU
    beyond (N = krk_set_digester_host_streams; -1 restores 40 x host CPUs)."""
    try:
        check(lib.krk_set_digester_host_streams(1 << 20))
        held = [core.NewDigester() for _ in range(3)]
        assert [d.placement() for d in held] == [KRK_PLACE_HOST] * 3
        check(lib.krk_set_digester_host_streams(0))
        g = core.NewDigester()
        assert g.placement() == KRK_PLACE_GPU
        for d in held + [g]:
            d._write(b"kraken")
            assert d.Digest().Hex() == hashlib.sha256(b"kraken").hexdigest()
    finally:
        check(lib.krk_set_digester_host_streams(-1))
    assert core.NewDigester().placement() == KRK_PLACE_HOST  # default: 40 x CPUs >> live digesters here


def _one_gpu_digester_rate(data: bytes) -> float:
    d = core.Digester(KRK_PLACE_GPU)
    t0 = time.perf_counter()
    for i in range(0, len(data), 1 << 20):
        d._write(data[i:i + (1 << 20)])
    dg = d.Digest()
    el = time.perf_counter() - t0
    assert dg.Hex() == hashlib.sha256(data).hexdigest()
    return len(data) / el


def test_256_concurrent_gpu_digesters(gpu):
    """256 digesters on 256 threads (16 MiB each, random write
    sizes), every digest equal to hashlib; their bytes are coalesced into multi-stream
    launches (> 8 streams a launch); creating a digester allocates nothing on the device
    (< 1 ms).  The rates are printed, not asserted: they are bench.py --workload engine's."""
    n, L = 256, 16 << 20
    rng = np.random.default_rng(256)
    base = rng.integers(0, 256, L + n * 4096, dtype=np.uint8).tobytes()
    datas = [memoryview(base)[i * 4096: i * 4096 + L] for i in range(n)]
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda m: hashlib.sha256(m).hexdigest(), datas))
    single = _one_gpu_digester_rate(bytes(datas[0]))  # also warms the engine and the slot pool
    # creation cost
    hs = [C.c_void_p() for _ in range(n)]
    t0 = time.perf_counter()
    for h in hs:
        check(lib.krk_digester_new_on(KRK_PLACE_GPU, C.byref(h)))
    create_ms = (time.perf_counter() - t0) * 1e3 / n
    for h in hs:
        lib.krk_digester_free(h)
    b0 = _stats()

    import threading
    bar = [threading.Barrier(n + 1)]

    def work(i):
        r = np.random.default_rng(i)
        d = core.Digester(KRK_PLACE_GPU)
        m, pos = datas[i], 0
        bar[0].wait()  # 256 uploads in progress at once: they start together
        while pos < L:
            k = min(L - pos, int(r.integers(1, 1 << 20)))
            d._write(m[pos:pos + k])
            pos += k
        return d.Digest().Hex()

    def run():
        bar[0] = threading.Barrier(n + 1)
        with ThreadPoolExecutor(n) as ex:
            futs = [ex.submit(work, i) for i in range(n)]
            bar[0].wait()  # the timed region starts when every thread holds its digester
            t0 = time.perf_counter()
            got = [f.result() for f in futs]
            return got, time.perf_counter() - t0

    assert run()[0] == want  # first round grows the pinned slot pool (one-time pinning)
    b0 = _stats()
    got, el = run()
    b1 = _stats()
    assert got == want
    agg = n * L / el
    jobs_per_launch = (b1[1] - b0[1]) / max(1, b1[0] - b0[0])
    print(f"single GPU digester {single / 1e6:.1f} MB/s; 256 concurrent {agg / 1e9:.2f} GB/s "
          f"({agg / n / 1e6:.1f} MB/s a stream, {agg / single:.0f}x); {jobs_per_launch:.1f} streams per SHA launch; "
          f"create {create_ms:.3f} ms")
    assert jobs_per_launch > 8  # (create_ms is printed, not asserted: no time in the parity gate)
    # (the rate from Python threads is capped by the GIL: their first requests trickle in
    # over ~70 ms; test_256_native_digesters measures the engine from native threads)


def test_256_native_digesters():
    """256 GPU Digesters on 256 native threads (tests/native/
    digesters.cpp, a C-ABI caller like the cgo layer), 16 MiB each in random writes of up to
    1 MiB: every digest equals the host SHA-256 of the same bytes and the requests of the
    256 owners share launches.  The aggregate rate (14.0-14.4 GB/s warm) is measured by
    bench.py --workload engine, not asserted here (no rate in the
    parity gate)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "digesters")
    assert os.path.exists(exe), "build() compiles tests/native"
    r = subprocess.run([exe, "256", "16", "3"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    rounds = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    print(rounds)
    assert len(rounds) == 3 and all(x["digests_match"] for x in rounds)
    assert all(x["streams_per_launch"] > 8 for x in rounds[1:]), rounds


@pytest.mark.parametrize("P", [3, 1000, 65536, 3 << 20, 5 << 20, 8 << 20])
def test_piece_stream_across_slots(gpu, P):
    """NewMetaInfo over a reader (calcPieceSums, core/metainfo.go:157-179) through the
    engine: pieces shorter and longer than a staging slot, a partial last piece, random
    read sizes; the portions of a piece that spans slots are combined on the host."""
    rng = np.random.default_rng(P)
    n = 3 * SLOT + 12345 if P < SLOT else 3 * P + 777
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()

    class Chunky(io.RawIOBase):
        def __init__(self, b):
            self.b, self.i = b, 0

        def read(self, k=-1):
            k = int(rng.integers(1, 3 << 20))
            out = self.b[self.i:self.i + k]
            self.i += len(out)
            return out

    length, sums = core.calcPieceSums(Chunky(data), P)
    assert length == n
    want = [zlib.crc32(data[i:i + P]) for i in range(0, n, P)]
    assert sums.tolist() == want


def test_crc32_update_host_and_queue(gpu):
    """crc32.Update semantics (seeded) for writes on both sides of the host crossover
    (<= 64 KiB on the caller's thread, larger through the CRC queue, multi-slot)."""
    rng = np.random.default_rng(7)
    for n in [0, 1, 4095, 65536, 65537, SLOT, SLOT + 1, 7 * SLOT + 3]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2 ** 32))
        out = C.c_uint32()
        check(lib.krk_crc32_update(seed, data, n, C.byref(out)))
        assert out.value == zlib.crc32(data, seed), n
        h = core.PieceHash()
        h.Write(data)
        h.Write(b"tail")
        assert h.Sum32() == zlib.crc32(data + b"tail"), n


def test_concurrent_streams_and_crc_share_launches(gpu):
    """Many threads: piece streams, crc32.Update and GPU digesters at once; results equal
    the serial reference and the CRC queue carried several requests per launch."""
    b0 = _stats()

    def work(i):
        r = np.random.default_rng(1000 + i)
        data = r.integers(0, 256, int(r.integers(SLOT, 4 * SLOT)), dtype=np.uint8).tobytes()
        P = int(r.choice([4096, 1 << 20, 3 << 20]))
        ok = core.calcPieceSums(io.BytesIO(data), P)[1].tolist() == [zlib.crc32(data[k:k + P])
                                                                     for k in range(0, len(data), P)]
        out = C.c_uint32()
        check(lib.krk_crc32_update(i, data, len(data), C.byref(out)))
        ok = ok and out.value == zlib.crc32(data, i)
        d = core.Digester(KRK_PLACE_GPU)
        d._write(data)
        return ok and d.Digest().Hex() == hashlib.sha256(data).hexdigest()

    with ThreadPoolExecutor(32) as ex:
        assert all(ex.map(work, range(64)))
    b1 = _stats()
    assert (b1[3] - b0[3]) > (b1[2] - b0[2])  # CRC requests per launch > 1
    assert b1[4] > 0  # pinned slot pool in use


def _run_script(code, env_extra, timeout=240):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # the engine's CRC side is what these scripts test: piece streams and crc32_update on
    # the GPU placement (a fresh process's AUTO would keep them on the caller's thread)
    env = dict(os.environ, KRK_CRC_PLACEMENT="2", **env_extra)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, cwd=root,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


_CAP_SCRIPT = r"""
import ctypes as C, hashlib, json, sys
from concurrent.futures import ThreadPoolExecutor
import numpy as np
sys.path.insert(0, ".")
from kraken_amd import core, device as D
from kraken_amd._capi import KRK_PLACE_GPU, check, lib
D.set_device(0)
n, L = 1024, 3 << 20
base = np.random.default_rng(1024).integers(0, 256, L + n * 512, dtype=np.uint8).tobytes()
datas = [memoryview(base)[i * 512: i * 512 + L] for i in range(n)]
digs = [core.Digester(KRK_PLACE_GPU) for _ in range(n)]
peak = [0]
def work(t):
    r = np.random.default_rng(t)
    mine = list(range(t, n, 64))
    pos = {i: 0 for i in mine}
    while pos:  # round-robin over this thread's 16 digesters, random write sizes
        for i in list(pos):
            k = min(L - pos[i], int(r.integers(1, 1 << 20)))
            digs[i]._write(datas[i][pos[i]:pos[i] + k])
            pos[i] += k
            if pos[i] == L:
                del pos[i]
        v = [C.c_uint64() for _ in range(5)]
        check(lib.krk_engine_stats(*[C.byref(x) for x in v]))
        peak[0] = max(peak[0], v[4].value)
    return [(i, digs[i].Digest().Hex()) for i in mine]
with ThreadPoolExecutor(64) as ex:
    got = dict(kv for part in ex.map(work, range(64)) for kv in part)
ok = all(got[i] == hashlib.sha256(datas[i]).hexdigest() for i in range(n))
cap, waits = C.c_uint64(), C.c_uint64()
check(lib.krk_engine_set_pool_cap(0, C.byref(cap), C.byref(waits)))
v = [C.c_uint64() for _ in range(5)]
check(lib.krk_engine_stats(*[C.byref(x) for x in v]))
print(json.dumps({"ok": ok, "cap": cap.value, "waits": waits.value, "pinned": v[4].value, "peak": peak[0],
                  "sha_batches": v[0].value, "sha_jobs": v[1].value}))
"""


def test_1024_digesters_under_hard_pool_cap(gpu):
    """VERDICT r02 item 10 / ADVICE: the slot pool's cap is hard.  1,024 GPU digesters
    (64 threads, 3 MiB each, random write sizes) under a 128 MiB cap (64 slots, far fewer
    than digesters x requests in flight): writers wait for slots instead of pinning more,
    pinned bytes never exceed the cap, and every digest equals hashlib."""
    import json
    out = _run_script(_CAP_SCRIPT, {"KRK_SLOT_POOL_MB": "128", "KRK_DIGESTER_HOST_STREAMS": "0"})
    d = json.loads(out.strip().splitlines()[-1])
    print(d)
    assert d["ok"] is True
    assert d["cap"] == 128 << 20
    assert d["pinned"] <= d["cap"] and d["peak"] <= d["cap"]
    assert d["waits"] > 0  # backpressure was exercised


_FAIL_SCRIPT = r"""
import ctypes as C, sys, zlib
import numpy as np
sys.path.insert(0, ".")
from kraken_amd import device as D
from kraken_amd._capi import check, lib, KrakenError
D.set_device(0)
rng = np.random.default_rng(7)
data = rng.integers(0, 256, 9 * (2 << 20) + 12345, dtype=np.uint8).tobytes()
P = 3 << 20 | 5  # pieces span slots: a failed slot leaves later portions with no start
s = C.c_void_p()
check(lib.krk_piece_stream_begin(P, C.byref(s)))
rc = 0
for i in range(0, len(data), 700001):
    chunk = data[i:i + 700001]
    rc = lib.krk_piece_stream_update(s, chunk, len(chunk))
    if rc:
        break
sums = (C.c_uint32 * 16)()
ns, ln = C.c_uint64(), C.c_uint64()
if not rc:
    rc = lib.krk_piece_stream_end(s, sums, 16, C.byref(ns), C.byref(ln))
msg = lib.krk_last_error().decode()
lib.krk_piece_stream_free(s)
# the engine keeps working after the failure
big = data[: 5 << 20]
out = C.c_uint32()
check(lib.krk_crc32_update(0, big, len(big), C.byref(out)))
print(rc, "|", msg, "|", out.value == zlib.crc32(big))
"""


def test_piece_stream_failure_mid_stream(gpu):
    """a CRC launch that fails in the middle of a piece stream
    (fault injected: the 2nd CRC launch of the engine) poisons the stream -- its later
    portions are not folded into sums the failed request never wrote -- and the error
    comes back from update/end; the engine serves later calls correctly."""
    from tests.conftest import diag_lib
    # fault injection is an A/B hook: the diag build reads it (knobs.hpp), production does not
    out = _run_script(_FAIL_SCRIPT, {"KRK_ENGINE_FAIL_CRC_LAUNCH": "2", "KRK_CRC_HOST_MAX": "1",
                                     "KRK_LIB_PATH": diag_lib()})
    rc, msg, ok = [x.strip() for x in out.strip().splitlines()[-1].split("|")]
    assert int(rc) != 0 and "injected failure" in msg, out
    assert ok == "True"
