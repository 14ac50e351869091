"""ctypes wrapper around the CPU oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- as the checker and the timed CPU baseline,
never as the product path.  See oracle.h for the parity status (pinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")


def build() -> str:
    """Compile liboracle.so (gcc, seconds)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def _load() -> C.CDLL:
    if not os.path.exists(_LIB_PATH):
        build()
    lib = C.CDLL(_LIB_PATH)
    u8p, u32p, u64p, i32p, i64p, f64p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int64), C.POINTER(C.c_double))
    sig = {
        "orc_crc32_update": (C.c_uint32, [C.c_uint32, C.c_void_p, C.c_uint64]),
        "orc_crc32_update_clmul": (C.c_uint32, [C.c_uint32, C.c_void_p, C.c_uint64]),
        "orc_have_clmul": (C.c_int, []),
        "orc_have_shani": (C.c_int, []),
        "orc_calc_piece_sums": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int64, u32p, u64p, u64p]),
        "orc_get_piece_length": (C.c_int64, [C.c_int64, C.c_int64, C.c_uint64, C.c_int64]),
        "orc_sha256": (None, [C.c_void_p, C.c_uint64, u8p]),
        "orc_sha256_shani": (None, [C.c_void_p, C.c_uint64, u8p]),
        "orc_sha1": (None, [C.c_void_p, C.c_uint64, u8p]),
        "orc_bencode_info": (C.c_uint64, [C.c_int64, u32p, C.c_uint64, C.c_char_p, C.c_uint64,
                                          C.c_int64, u8p, C.c_uint64]),
        "orc_info_hash": (None, [C.c_int64, u32p, C.c_uint64, C.c_char_p, C.c_uint64, C.c_int64, u8p]),
        "orc_murmur3_h1": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_uint64]),
        "orc_go_log": (C.c_double, [C.c_double]),
        "orc_uint64_to_float64": (C.c_double, [C.c_uint64, C.c_int]),
        "orc_hrw_score": (C.c_double, [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, C.c_int64]),
        "orc_hrw_ordered": (C.c_int, [C.c_char_p, C.c_uint64, C.c_char_p, u64p, i64p, C.c_uint32,
                                      C.c_uint32, i32p, f64p]),
        "orc_ring_locations": (C.c_uint32, [i32p, C.c_uint32, u8p, C.c_int32, i32p]),
        "orc_ring_owner_table": (None, [C.c_char_p, u64p, i64p, C.c_uint32, u8p, C.c_int32, C.c_uint32, i32p,
                                        u8p]),
        "orc_piece_length_for_size": (C.c_int64, [i64p, i64p, C.c_uint32, C.c_int64]),
        "orc_blob_seed": (C.c_uint64, [C.c_uint64]),
        "orc_synth_fill": (None, [C.c_uint64, C.c_uint64, u8p, C.c_uint64, C.c_int]),
        "orc_baseline_run": (C.c_double, [u64p, u64p, C.c_uint64, C.c_int64, C.c_int, C.c_int, C.c_int,
                                          C.c_uint64, u8p, u32p, u64p]),
        "orc_baseline_files": (C.c_double, [C.POINTER(C.c_char_p), u64p, C.c_uint64, C.c_int64, C.c_int, C.c_int,
                                            u32p, u64p, u8p]),
        "orc_crc_bufs": (C.c_double, [C.POINTER(C.c_void_p), u64p, C.c_uint64, C.c_int, u32p]),
        "orc_baseline_run_lazy": (C.c_double, [u64p, u64p, C.c_uint64, C.c_int64, C.c_int, C.c_int,
                                               u8p, u32p, u64p]),
        "orc_baseline_hrw": (C.c_double, [u8p, C.c_uint64, C.c_char_p, u64p, C.c_uint32, u8p,
                                          C.c_int32, C.c_int, i32p, u8p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


def _buf(data) -> tuple:
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None)


# ---- CRC / pieces -------------------------------------------------------

def crc32(data, crc: int = 0) -> int:
    a, p = _buf(data)
    return lib().orc_crc32_update(crc, p, a.size)


def crc32_clmul(data, crc: int = 0) -> int:
    a, p = _buf(data)
    return lib().orc_crc32_update_clmul(crc, p, a.size)


def calc_piece_sums(data, piece_length: int):
    """core.calcPieceSums (core/metainfo.go:158-179) -> (length, [sums])."""
    a, p = _buf(data)
    n = C.c_uint64()
    ln = C.c_uint64()
    if lib().orc_calc_piece_sums(p, a.size, piece_length, None, C.byref(n), C.byref(ln)) != 0:
        raise ValueError("piece length must be positive")
    out = np.zeros(max(n.value, 1), dtype=np.uint32)
    lib().orc_calc_piece_sums(p, a.size, piece_length, _ptr(out, C.c_uint32), C.byref(n), C.byref(ln))
    return ln.value, out[: n.value]


def get_piece_length(length: int, piece_length: int, n_pieces: int, i: int) -> int:
    return lib().orc_get_piece_length(length, piece_length, n_pieces, i)


# ---- digests ------------------------------------------------------------

def sha256(data) -> bytes:
    a, p = _buf(data)
    out = (C.c_uint8 * 32)()
    lib().orc_sha256(p, a.size, out)
    return bytes(out)


def sha256_shani(data) -> bytes:
    a, p = _buf(data)
    out = (C.c_uint8 * 32)()
    lib().orc_sha256_shani(p, a.size, out)
    return bytes(out)


def sha1(data) -> bytes:
    a, p = _buf(data)
    out = (C.c_uint8 * 20)()
    lib().orc_sha1(p, a.size, out)
    return bytes(out)


def bencode_info(piece_length: int, sums, name: str, length: int) -> bytes:
    s = np.ascontiguousarray(np.asarray(sums, dtype=np.uint32))
    sp = _ptr(s, C.c_uint32) if s.size else None
    nb = name.encode()
    need = lib().orc_bencode_info(piece_length, sp, s.size, nb, len(nb), length, None, 0)
    out = (C.c_uint8 * need)()
    lib().orc_bencode_info(piece_length, sp, s.size, nb, len(nb), length, out, need)
    return bytes(out)


def info_hash(piece_length: int, sums, name: str, length: int) -> bytes:
    s = np.ascontiguousarray(np.asarray(sums, dtype=np.uint32))
    sp = _ptr(s, C.c_uint32) if s.size else None
    nb = name.encode()
    out = (C.c_uint8 * 20)()
    lib().orc_info_hash(piece_length, sp, s.size, nb, len(nb), length, out)
    return bytes(out)


# ---- HRW ----------------------------------------------------------------

def murmur3_h1(data, seed: int = 0) -> int:
    a, p = _buf(data)
    return lib().orc_murmur3_h1(p, a.size, seed)


def go_log(x: float) -> float:
    return lib().orc_go_log(x)


def uint64_to_float64(h1: int, rehash: bool = True) -> float:
    return lib().orc_uint64_to_float64(h1, 1 if rehash else 0)


def hrw_score(key_hex: str, label: str, weight: int) -> float:
    k, l = key_hex.encode(), label.encode()
    return lib().orc_hrw_score(k, len(k), l, len(l), weight)


def _labels(labels):
    enc = [s.encode() for s in labels]
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(e) for e in enc]) if enc else []
    return b"".join(enc), off


def hrw_ordered(key_hex: str, labels, weights, n: int | None = None, with_scores=False):
    """GetOrderedNodes(key, n) -> list of node indices (and scores)."""
    blob, off = _labels(labels)
    w = np.ascontiguousarray(np.asarray(weights, dtype=np.int64))
    N = len(labels)
    n = N if n is None else n
    order = np.zeros(max(N, 1), dtype=np.int32)
    scores = np.zeros(max(N, 1), dtype=np.float64)
    k = key_hex.encode()
    m = lib().orc_hrw_ordered(k, len(k), blob, _ptr(off, C.c_uint64), _ptr(w, C.c_int64), N, n,
                              _ptr(order, C.c_int32), _ptr(scores, C.c_double))
    if with_scores:
        return order[:m].tolist(), scores[:N].tolist()
    return order[:m].tolist()


def ring_locations(order, healthy, max_replica: int):
    o = np.ascontiguousarray(np.asarray(order, dtype=np.int32))
    h = np.ascontiguousarray(np.asarray(healthy, dtype=np.uint8))
    out = np.zeros(max(len(order), 1), dtype=np.int32)
    k = lib().orc_ring_locations(_ptr(o, C.c_int32), len(order), _ptr(h, C.c_uint8), max_replica,
                                 _ptr(out, C.c_int32))
    return out[:k].tolist()


def ring_owner_table(labels, weights, healthy, max_replica: int):
    """Every ShardID's Locations (65,536 rows, -1 padded to max(1, max_replica)) and counts."""
    blob, off = _labels(labels)
    w = np.ascontiguousarray(np.asarray(weights, dtype=np.int64))
    h = np.ascontiguousarray(np.asarray(healthy, dtype=np.uint8))
    row = max(1, int(max_replica))
    locs = np.zeros((65536, row), dtype=np.int32)
    counts = np.zeros(65536, dtype=np.uint8)
    lib().orc_ring_owner_table(blob, _ptr(off, C.c_uint64), _ptr(w, C.c_int64), len(labels), _ptr(h, C.c_uint8),
                               int(max_replica), row, _ptr(locs, C.c_int32), _ptr(counts, C.c_uint8))
    return locs, counts


def piece_length_for_size(ranges: dict, size: int) -> int:
    items = sorted(ranges.items())
    t = np.array([a for a, _ in items], dtype=np.int64)
    l = np.array([b for _, b in items], dtype=np.int64)
    return lib().orc_piece_length_for_size(_ptr(t, C.c_int64), _ptr(l, C.c_int64), len(items), size)


# ---- synthetic content ----------------------------------------------------

def blob_seed(i: int) -> int:
    return lib().orc_blob_seed(i)


def synth(blob_idx: int, length: int, offset: int = 0, variant: int = 0) -> np.ndarray:
    out = np.empty(length, dtype=np.uint8)
    if length:
        lib().orc_synth_fill(blob_idx, offset, _ptr(out, C.c_uint8), length, variant)
    return out


# ---- CPU baseline -----------------------------------------------------------

def baseline_run(blob_idx, lengths, piece_length: int, threads: int, fast: bool = True,
                 want_outputs: bool = False, repeats: int = 1, passes: int = 3):
    """Times the reference's two-pass structure (SHA pass, then CRC piece pass),
    one blob per worker thread.  Returns (seconds, digests|None, sums|None)."""
    bi = np.ascontiguousarray(np.asarray(blob_idx, dtype=np.uint64))
    ln = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    dg = sums = off = None
    dp = sp = op = None
    if want_outputs:
        dg = np.zeros((len(bi), 32), dtype=np.uint8)
        npieces = [(int(l) + piece_length - 1) // piece_length for l in ln]
        off = np.zeros(len(bi) + 1, dtype=np.uint64)
        off[1:] = np.cumsum(npieces)
        sums = np.zeros(max(int(off[-1]), 1), dtype=np.uint32)
        dp, sp, op = _ptr(dg, C.c_uint8), _ptr(sums, C.c_uint32), _ptr(off, C.c_uint64)
    t = lib().orc_baseline_run(_ptr(bi, C.c_uint64), _ptr(ln, C.c_uint64), len(bi), piece_length,
                               threads, 1 if fast else 0, passes, repeats, dp, sp, op)
    return t, dg, (sums, off) if want_outputs else None


def baseline_run_lazy(blob_idx, lengths, piece_length: int, threads: int, passes: int = 3):
    """orc_baseline_run_lazy: one buffer per thread, each blob generated untimed before
    its passes.  Returns (summed busy seconds, digests, (sums, offsets))."""
    bi = np.ascontiguousarray(np.asarray(blob_idx, dtype=np.uint64))
    ln = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    dg = np.zeros((len(bi), 32), dtype=np.uint8)
    npieces = [(int(l) + piece_length - 1) // piece_length for l in ln]
    off = np.zeros(len(bi) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(npieces)
    sums = np.zeros(max(int(off[-1]), 1), dtype=np.uint32)
    busy = lib().orc_baseline_run_lazy(_ptr(bi, C.c_uint64), _ptr(ln, C.c_uint64), len(bi), piece_length, threads,
                                       passes, _ptr(dg, C.c_uint8), _ptr(sums, C.c_uint32), _ptr(off, C.c_uint64))
    return busy, dg, (sums, off)


def crc_bufs(ptrs, lengths, threads: int):
    """orc_crc_bufs: one CRC-32 per caller buffer (addresses `ptrs`, byte counts `lengths`) on
    `threads` threads.  Returns (seconds, sums)."""
    n = len(ptrs)
    pa = (C.c_void_p * max(n, 1))(*[int(x) for x in ptrs])
    ln = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    sums = np.zeros(max(n, 1), dtype=np.uint32)
    t = lib().orc_crc_bufs(pa, _ptr(ln, C.c_uint64), n, threads, _ptr(sums, C.c_uint32))
    return t, sums[:n]


def baseline_files(paths, lengths, piece_length: int, threads: int, passes: int = 2):
    """orc_baseline_files: the reference's passes over CAS files on `threads` threads --
    passes & 1 the upload verify (Digester over the file, 32 KiB reads), passes & 2 Generate
    (calcPieceSums over the file reader).  Returns (seconds, sums, offsets), plus the
    digests when passes & 1."""
    n = len(paths)
    enc = (C.c_char_p * max(n, 1))(*[p.encode() if isinstance(p, str) else p for p in paths])
    ln = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    npieces = [(int(l) + piece_length - 1) // piece_length for l in ln]
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(npieces)
    sums = np.zeros(max(int(off[-1]), 1), dtype=np.uint32)
    dg = np.zeros((max(n, 1), 32), dtype=np.uint8)
    t = lib().orc_baseline_files(enc, _ptr(ln, C.c_uint64), n, piece_length, threads, passes,
                                 _ptr(sums, C.c_uint32), _ptr(off, C.c_uint64), _ptr(dg, C.c_uint8))
    if t < 0:
        raise OSError("orc_baseline_files: a file could not be read to its length")
    return (t, sums, off, dg[:n]) if passes & 1 else (t, sums, off)


def baseline_hrw(digests: np.ndarray, labels, healthy, max_replica: int, threads: int):
    d = np.ascontiguousarray(digests, dtype=np.uint8)
    n = d.shape[0]
    blob, off = _labels(labels)
    h = np.ascontiguousarray(np.asarray(healthy, dtype=np.uint8))
    mo = max(1, max_replica)
    locs = np.zeros((n, mo), dtype=np.int32)
    counts = np.zeros(n, dtype=np.uint8)
    t = lib().orc_baseline_hrw(_ptr(d, C.c_uint8), n, blob, _ptr(off, C.c_uint64), len(labels),
                               _ptr(h, C.c_uint8), max_replica, threads, _ptr(locs, C.c_int32),
                               _ptr(counts, C.c_uint8))
    return t, locs, counts
