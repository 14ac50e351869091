"""GPU parity: batched agent piece verification (agentstorage.Torrent.writePiece,
lib/torrent/storage/agentstorage/torrent.go:174-220) through krk_verify_pieces_host,
against zlib.crc32 (= Go hash/crc32 IEEE) and the reference's error strings."""
import io
import os
import zlib

import numpy as np
import pytest

from kraken_amd import agentstorage, core

pytestmark = pytest.mark.gpu


def test_verify_pieces_matches_crc32(gpu):
    rng = np.random.default_rng(11)
    lens = [0, 1, 2, 3, 4, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 262143, 262144, 262145,
            (1 << 20) + 1, 4 << 20, (4 << 20) - 3]
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    expected = [zlib.crc32(d) for d in datas]
    assert agentstorage.verify_pieces(datas, expected).all()
    # one flipped bit / one wrong sum per piece -> every check fails
    bad = [bytes([d[0] ^ 1]) + d[1:] if d else d for d in datas]
    ok = agentstorage.verify_pieces(bad, expected)
    assert ok.tolist() == [len(d) == 0 for d in datas]
    ok = agentstorage.verify_pieces(datas, [e ^ 0x80000000 for e in expected])
    assert not ok.any()


def test_verify_many_small_pieces_one_call(gpu):
    rng = np.random.default_rng(12)
    datas = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 5000, 3000)]
    expected = np.array([zlib.crc32(d) for d in datas], dtype=np.uint32)
    flip = rng.choice(len(datas), 100, replace=False)
    expected[flip] ^= 1
    ok = agentstorage.verify_pieces(datas, expected)
    want = np.ones(len(datas), dtype=bool)
    want[flip] = False
    assert np.array_equal(ok, want)


def test_torrent_write_pieces(gpu, tmp_path):
    rng = np.random.default_rng(13)
    blob = rng.integers(0, 256, size=10 * 65536 + 1234, dtype=np.uint8).tobytes()
    P = 65536
    d = core.NewDigester().FromBytes(blob)
    mi = core.NewMetaInfo(d, io.BytesIO(blob), P)
    t = agentstorage.Torrent(mi, str(tmp_path / "download"))
    pieces = {pi: blob[pi * P:pi * P + mi.GetPieceLength(pi)] for pi in range(mi.NumPieces())}
    corrupt = dict(pieces)
    corrupt[3] = b"\x00" + pieces[3][1:]
    first = {pi: corrupt[pi] for pi in (7, 3, 10, 0)}
    res = t.WritePieces(first)
    assert res[7] is None and res[10] is None and res[0] is None
    assert str(res[3]) == "invalid piece sum"
    with pytest.raises(ValueError, match="invalid piece length: expected 65536, got 3"):
        t.WritePiece(b"abc", 5)
    with pytest.raises(agentstorage.ErrPieceComplete):
        t.WritePiece(pieces[7], 7)
    rest = {pi: pieces[pi] for pi in range(mi.NumPieces()) if not t.complete[pi]}
    assert all(e is None for e in t.WritePieces(rest).values())
    assert t.Complete()
    assert open(tmp_path / "download", "rb").read() == blob


@pytest.mark.parametrize("frac", ["auto", "0", "0.5", "1"])
@pytest.mark.parametrize("pinned", [True, False])
def test_host_gpu_split_bit_exact(gpu, monkeypatch, frac, pinned):
    """krk_piece_sums_host / krk_verify_pieces_host split a batch
    between host PCLMUL threads and the GPU pass (pinned caller bytes: DMA straight into
    the device window) by the measured rates; every split -- all host, half, all GPU,
    the planner's own -- gives zlib's sums and the same verdicts, for pieces of ragged
    lengths in pinned and pageable memory, and multi-piece blobs split mid-blob."""
    from kraken_amd import device as D
    if frac != "auto":
        monkeypatch.setenv("KRK_CRC_GPU_FRACTION", frac)
    rng = np.random.default_rng(99)
    lens = [int(x) for x in rng.integers(1, 3 << 20, 200)] + [0, 1, 4 << 20]
    total = sum(lens)
    if pinned:
        buf = D.PinnedArray((total,), np.uint8)
        arr = buf.a
    else:
        arr = np.empty(total, dtype=np.uint8)
    arr[:] = rng.integers(0, 256, total, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    datas = [arr[offs[i]:offs[i + 1]] for i in range(len(lens))]
    expected = np.array([zlib.crc32(d.tobytes()) for d in datas], dtype=np.uint32)
    flip = rng.choice(len(lens), 20, replace=False)
    exp = expected.copy()
    exp[flip] ^= 0x10
    want = np.ones(len(lens), dtype=bool)
    want[flip] = False
    assert np.array_equal(agentstorage.verify_pieces(datas, exp), want)
    # multi-piece blobs (64 KiB + 3 B pieces): the split may cut a blob between pieces
    P = (64 << 10) + 3
    big = [arr[: 40 * P + 17], arr[5: 5 + 7 * P]]
    for b, s in zip(big, D.piece_sums_host(big, P)):
        want_s = [zlib.crc32(b[k:k + P].tobytes()) for k in range(0, b.size, P)]
        assert [int(x) for x in s] == want_s


def _place_stripes(arr, stripe):
    """Moves the pages of `arr` (page-aligned) to NUMA nodes 0 and 1 in alternating stripes of
    `stripe` bytes (move_pages(2)); False when the host has one node or the call fails."""
    import ctypes
    nodes = [d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")] \
        if os.path.isdir("/sys/devices/system/node") else []
    if len(nodes) < 2:
        return False
    libc = ctypes.CDLL(None, use_errno=True)
    n = arr.size // 4096
    pages = (ctypes.c_void_p * n)(*[arr.ctypes.data + i * 4096 for i in range(n)])
    dst = (ctypes.c_int * n)(*[(i * 4096 // stripe) & 1 for i in range(n)])
    status = (ctypes.c_int * n)()
    return libc.syscall(279, 0, ctypes.c_ulong(n), pages, dst, status, 2) == 0  # SYS_move_pages, MPOL_MF_MOVE


_NUMA_SCRIPT = r"""
import mmap, sys, zlib
import numpy as np
sys.path.insert(0, sys.argv[1])
from tests.test_gpu_agent_verify import _place_stripes
from kraken_amd import device as D
D.set_device(0)
P, L = 256 << 10, 192 << 20
for shift in (0, 4 << 20):
    m = mmap.mmap(-1, L)
    arr = np.frombuffer(m, dtype=np.uint8)
    arr[:] = np.random.default_rng(7).integers(0, 256, L, dtype=np.uint8)
    _place_stripes(arr, 8 << 20)
    blob = arr[shift:]
    (s,) = D.piece_sums_host([blob], P)
    want = [zlib.crc32(blob[k:k + P].tobytes()) for k in range(0, blob.size, P)]
    assert [int(x) for x in s] == want, shift
    del arr, blob, s
    m.close()
print("ok")
"""


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_host_crc_numa_handout_bit_exact(gpu, mode):
    """The host CRC share's NUMA-aware hand-out (KRK_CRC_NUMA: 0 one cursor, the default; 1
    per-node claims; 2 per-node claims + node visits) over a buffer whose 8 MiB runs sit on
    alternating nodes (and on a half-stripe offset, so every task straddles two nodes and is
    never visited): every task is summed once, the sums are zlib's.  KRK_CRC_NUMA is an A/B
    switch (knobs.hpp): the diag build reads it, once a process, so each mode runs in a fresh
    process on that build."""
    import subprocess
    import sys
    from tests.conftest import ROOT, diag_lib
    env = dict(os.environ, KRK_CRC_NUMA=mode, KRK_CRC_GPU_FRACTION="0",  # every byte through the host hand-out
               KRK_LIB_PATH=diag_lib())
    r = subprocess.run([sys.executable, "-c", _NUMA_SCRIPT, ROOT], capture_output=True, text=True, timeout=240,
                       cwd=ROOT, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
