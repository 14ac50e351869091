"""Device-resident batch helpers over the C ABI (used by bench.py and the GPU
parity tests): an HBM arena of synthetic blobs and the batch calls on it."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, krk_blob, krk_file_blob, krk_chunk, krk_launch_rec, krk_nodes, krk_planner_rates, lib

ALIGN = 256  # every blob starts 256-byte aligned in the arena


class DeviceBuffer:
    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib.krk_dev_alloc(max(int(nbytes), 1), C.byref(p)))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    def free(self):
        if self.ptr:
            lib.krk_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def to_host(self, dtype=np.uint8, count: int | None = None, offset: int = 0) -> np.ndarray:
        it = np.dtype(dtype).itemsize
        n = (self.nbytes - offset) // it if count is None else count
        out = np.empty(n, dtype=dtype)
        if n:
            check(lib.krk_memcpy_d2h(out.ctypes.data, self.ptr + offset, n * it))
        return out

    def zero(self):
        self.from_host(np.zeros(self.nbytes, dtype=np.uint8))

    def from_host(self, a: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(a)
        if a.nbytes:
            check(lib.krk_memcpy_h2d(self.ptr + offset, a.ctypes.data, a.nbytes))


class PinnedArray:
    """A numpy view of library-allocated pinned host memory (krk_host_alloc):
    device results land here at PCIe rate instead of through a pageable bounce."""

    def __init__(self, shape, dtype, dma_target=False):
        """dma_target: the HIP runtime's allocator (krk_host_alloc_dma: the device's NUMA
        node) for buffers the device copies into."""
        self.array_nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = C.c_void_p()
        check((lib.krk_host_alloc_dma if dma_target else lib.krk_host_alloc)(max(self.array_nbytes, 1), C.byref(p)))
        self.ptr = p.value
        buf = (C.c_uint8 * max(self.array_nbytes, 1)).from_address(self.ptr)
        self.a = np.frombuffer(buf, dtype=np.uint8, count=self.array_nbytes).view(dtype).reshape(shape)

    def fill_from(self, dev: "DeviceBuffer", offset: int = 0):
        if self.array_nbytes:
            check(lib.krk_memcpy_d2h(self.ptr, dev.ptr + offset, self.array_nbytes))
        return self.a

    def fill_from_async(self, dev: "DeviceBuffer", stream, offset: int = 0):
        """Queue the copy on `stream`; self.a is valid once that stream is synchronised."""
        if self.array_nbytes:
            check(lib.krk_memcpy_d2h_async(self.ptr, dev.ptr + offset, self.array_nbytes, stream))

    def __del__(self):
        try:
            if self.ptr:
                lib.krk_host_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


def device_count() -> int:
    n = C.c_int()
    check(lib.krk_device_count(C.byref(n)))
    return n.value


def set_device(d: int):
    check(lib.krk_set_device(d))


def init(dev_mask: int = 0):
    """Create device contexts eagerly (krk_init): bit i = device i, 0 = current."""
    check(lib.krk_init(dev_mask))


def shutdown():
    """Free every device context and the pinned staging windows (krk_shutdown).
    No library call may be in flight; later calls re-create contexts lazily."""
    check(lib.krk_shutdown())


def synchronize():
    check(lib.krk_synchronize())


def sha_lanes_per_stream(n_streams: int) -> int:
    """Lanes per SHA-256 stream the library uses for a batch of n_streams (1, 2 or 8)."""
    v = C.c_int(0)
    check(lib.krk_sha_lanes_per_stream(n_streams, C.byref(v)))
    return v.value


SHA_PLAN_NAMES = {1: "1lane", 2: "2lane", 3: "1lane_2pair", 4: "2lane_2pair", 5: "8lane", 6: "8lane_2pair"}


def sha_plan_for(n_streams: int) -> int:
    """KRK_SHA_PLAN_* id the library launches for a batch of n_streams (SHA_PLAN_NAMES)."""
    v = C.c_int(0)
    check(lib.krk_sha_plan_for(n_streams, C.byref(v)))
    return v.value


KRK_BLOB_DTYPE = np.dtype([("data", "<u8"), ("length", "<u8"), ("piece_length", "<i8"), ("sums_offset", "<u8")])
assert KRK_BLOB_DTYPE.itemsize == C.sizeof(krk_blob)


class BlobArena:
    """Blobs laid out back to back in one HBM allocation (each 256 B aligned)."""

    def __init__(self, lengths, piece_length, blob_ids=None, variant: int = 0, fill: bool = True,
                 misalign: int = 0):
        self.lengths = np.asarray(lengths, dtype=np.uint64)
        n = len(self.lengths)
        pls = np.broadcast_to(np.asarray(piece_length, dtype=np.int64), (n,))
        self.piece_lengths = np.array(pls, dtype=np.int64)
        self.blob_ids = np.arange(n, dtype=np.uint64) if blob_ids is None else np.asarray(blob_ids, np.uint64)
        self.offsets = np.zeros(n, dtype=np.uint64)
        o = 0
        for i, L in enumerate(self.lengths):
            self.offsets[i] = o + misalign  # misalign > 0 exercises the unaligned path
            o += (int(L) + misalign + ALIGN - 1) // ALIGN * ALIGN
        self.nbytes = max(o, 1)
        self.buf = DeviceBuffer(self.nbytes)
        self.n_pieces = np.array([lib.krk_num_pieces(int(L), int(p)) for L, p in
                                  zip(self.lengths, self.piece_lengths)], dtype=np.uint64)
        self.sums_off = np.zeros(n, dtype=np.uint64)
        if n:
            self.sums_off[1:] = np.cumsum(self.n_pieces)[:-1]
        self.total_pieces = int(self.n_pieces.sum())
        if fill:
            for i in range(n):
                self.fill(i, variant)
            synchronize()

    def fill(self, i: int, variant: int = 0):
        check(lib.krk_synth_fill_dev(self.buf.ptr + int(self.offsets[i]), int(self.blob_ids[i]), 0,
                                     int(self.lengths[i]), variant, None))

    def put(self, i: int, data: np.ndarray):
        self.buf.from_host(np.asarray(data, dtype=np.uint8), int(self.offsets[i]))

    def blob_structs(self):
        """krk_blob[] of the arena, built once (column-wise) and cached: the layout
        never changes after construction."""
        arr = getattr(self, "_structs", None)
        if arr is None:
            n = len(self.lengths)
            a = np.zeros(max(n, 1), dtype=KRK_BLOB_DTYPE)
            a["data"][:n] = np.uint64(self.buf.ptr) + self.offsets
            a["length"][:n], a["piece_length"][:n], a["sums_offset"][:n] = \
                self.lengths, self.piece_lengths, self.sums_off
            arr = (krk_blob * max(n, 1)).from_buffer_copy(a.tobytes())
            self._structs = arr
        return arr

    def data_ptrs(self):
        n = len(self.lengths)
        ptrs = (C.c_void_p * max(n, 1))(*[self.buf.ptr + int(o) for o in self.offsets])
        lens = np.ascontiguousarray(self.lengths, dtype=np.uint64)
        return ptrs, lens


class BatchOutputs:
    def __init__(self, arena: BlobArena):
        self.sums = DeviceBuffer(max(arena.total_pieces, 1) * 4)
        self.digests = DeviceBuffer(max(len(arena.lengths), 1) * 32)


def piece_sums(arena: BlobArena, out: BatchOutputs, stream=None):
    check(lib.krk_piece_sums_dev(arena.blob_structs(), len(arena.lengths), out.sums.ptr, stream))


def pack_names(names):
    """The (bytes, offsets) layout krk_metainfo_batch_dev takes for the blobs' names."""
    enc = [x.encode() for x in names]
    noff = np.zeros(len(enc) + 1, dtype=np.uint64)
    noff[1:] = np.cumsum([len(e) for e in enc]) if enc else []
    return b"".join(enc), noff


def metainfo_batch(arena: BlobArena, out: BatchOutputs, names, sums_host: np.ndarray, stream=None) -> np.ndarray:
    """Generator.Generate over the arena's blobs (krk_metainfo_batch_dev): piece sums into
    out.sums and sums_host (uint32, arena layout) and the InfoHashes, returned as an
    (n, 20) uint8 array; the host hashes each group while later groups' kernels run.
    names: the blobs' names (str), or pack_names() of them."""
    n = len(arena.lengths)
    buf, noff = names if isinstance(names, tuple) else pack_names(names)
    if noff.size != n + 1:
        raise ValueError(f"metainfo_batch: {noff.size - 1} names for {n} blobs")
    ih = np.zeros((max(n, 1), 20), dtype=np.uint8)
    assert sums_host.dtype == np.uint32 and sums_host.size >= arena.total_pieces
    check(lib.krk_metainfo_batch_dev(arena.blob_structs(), n, buf or None,
                                     noff.ctypes.data_as(C.POINTER(C.c_uint64)), out.sums.ptr,
                                     sums_host.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     ih.ctypes.data_as(C.POINTER(C.c_uint8)), stream))
    return ih[:n]


def sha256(arena: BlobArena, out: BatchOutputs, stream=None):
    ptrs, lens = arena.data_ptrs()
    check(lib.krk_sha256_dev(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), len(arena.lengths),
                             out.digests.ptr, stream))


def sha256_dev_on_host(ptrs, lens, threads: int = 0, stream=None) -> np.ndarray:
    """krk_sha256_dev_on_host: device blobs (numpy device addresses + lengths) hashed by
    up to `threads` host threads after `stream`'s queued work; (n, 32) uint8 digests."""
    n = len(ptrs)
    p = np.ascontiguousarray(ptrs, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros((max(n, 1), 32), dtype=np.uint8)
    check(lib.krk_sha256_dev_on_host(p.ctypes.data_as(C.POINTER(C.c_void_p)), ln.ctypes.data_as(C.POINTER(C.c_uint64)),
                                     n, int(threads), stream, out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out[:n]


def piece_sums_dev_arrays(ptrs, lens, piece_lengths, sums_offsets, sums_dev_ptr: int, stream=None):
    """krk_piece_sums_dev over blobs given column-wise (device addresses, lengths, piece
    lengths, offsets of their sums in the sums buffer at sums_dev_ptr)."""
    n = len(ptrs)
    a = np.zeros(max(n, 1), dtype=KRK_BLOB_DTYPE)
    a["data"][:n], a["length"][:n] = ptrs, lens
    a["piece_length"][:n], a["sums_offset"][:n] = piece_lengths, sums_offsets
    check(lib.krk_piece_sums_dev(a.ctypes.data_as(C.POINTER(krk_blob)), n, sums_dev_ptr, stream))


def metainfo_digest(arena: BlobArena, out: BatchOutputs, stream=None):
    check(lib.krk_metainfo_digest_dev(arena.blob_structs(), len(arena.lengths), out.sums.ptr,
                                      out.digests.ptr, stream))


def set_sha_host_offload(threads: int):
    """krk_set_sha_host_offload: up to `threads` host threads take the longest SHA-256
    chains of sha256 / metainfo_digest batches (0 = off; -1 = AUTO, the default: the
    planner-gated offload on the process's CPU budget)."""
    check(lib.krk_set_sha_host_offload(int(threads)))


OFFLOAD_DEVICE, OFFLOAD_HOST_SHA, OFFLOAD_HOST_WHOLE, OFFLOAD_HOST_FILES = 0, 1, 2, 3


def piece_sums_host(datas, piece_length: int):
    """krk_piece_sums_host over host buffers (numpy uint8 arrays or bytes): each one's
    piece sums (calcPieceSums), split between host threads and the GPU by the planner."""
    arrs = [np.frombuffer(d, dtype=np.uint8) if isinstance(d, (bytes, bytearray)) else d for d in datas]
    n = len(arrs)
    blobs = (krk_blob * max(n, 1))()
    off = 0
    counts = []
    for i, a in enumerate(arrs):
        cnt = int(lib.krk_num_pieces(int(a.size), int(piece_length)))
        blobs[i] = krk_blob(a.ctypes.data if a.size else None, int(a.size), int(piece_length), off)
        counts.append(cnt)
        off += cnt
    sums = np.zeros(max(off, 1), dtype=np.uint32)
    check(lib.krk_piece_sums_host(blobs, n, sums.ctypes.data_as(C.POINTER(C.c_uint32))))
    out, o = [], 0
    for c in counts:
        out.append(sums[o:o + c].copy())
        o += c
    return out


def crc_host_split():
    """(GPU bytes, host bytes) of this thread's last krk_piece_sums_host / verify call and
    the GPU share the next pinned batch will use (-1 until learned)."""
    g, h, f = C.c_uint64(), C.c_uint64(), C.c_double()
    check(lib.krk_crc_host_split(C.byref(g), C.byref(h), C.byref(f)))
    return g.value, h.value, f.value


RATES_SOURCE = {0: "nominal", 1: "measured", 2: "set"}


def planner_rates() -> dict:
    """krk_planner_rates_get: the rates the planners use on this thread's device
    (measured there at first use; nominal without a device; or what was set)."""
    r = krk_planner_rates()
    check(lib.krk_planner_rates_get(C.byref(r)))
    return {"sha_stream_bps": list(r.sha_stream_bps), "d2h_bps": r.d2h_bps, "h2d_bps": r.h2d_bps,
            "host_sha_bps": r.host_sha_bps, "host_crc_bps": r.host_crc_bps, "host_copy_bps": r.host_copy_bps,
            "cus": r.cus,
            "source": RATES_SOURCE.get(r.source, r.source)}


def set_planner_rates(rates: dict | None):
    """krk_planner_rates_set (None: back to the measured / nominal rates)."""
    if rates is None:
        check(lib.krk_planner_rates_set(None))
        return
    r = krk_planner_rates()
    for k, v in enumerate(rates["sha_stream_bps"]):
        r.sha_stream_bps[k] = v
    r.d2h_bps, r.h2d_bps = rates["d2h_bps"], rates["h2d_bps"]
    r.host_sha_bps, r.host_crc_bps = rates["host_sha_bps"], rates["host_crc_bps"]
    r.host_copy_bps = rates["host_copy_bps"]
    r.cus = rates["cus"]
    check(lib.krk_planner_rates_set(C.byref(r)))


def sha_tail_plan(lengths, threads: int):
    """krk_sha_tail_plan: (chain indices whose tails host threads finish, the GPU's prefix
    bytes of each, planned end seconds, GPU-alone seconds) -- planner_rates(), no device."""
    L = np.ascontiguousarray(lengths, dtype=np.uint64)
    idx = np.zeros(max(L.size, 1), dtype=np.uint32)
    st = np.zeros(max(L.size, 1), dtype=np.uint64)
    k, e, g = C.c_uint64(0), C.c_double(0), C.c_double(0)
    check(lib.krk_sha_tail_plan(L.ctypes.data_as(C.POINTER(C.c_uint64)), L.size, int(threads),
                                idx.ctypes.data_as(C.POINTER(C.c_uint32)), st.ctypes.data_as(C.POINTER(C.c_uint64)),
                                C.byref(k), C.byref(e), C.byref(g)))
    return idx[:k.value].copy(), st[:k.value].copy(), e.value, g.value


def sha_last_tail() -> dict:
    """krk_sha_last_tail: the calling thread's last device-resident SHA-256 batch's tail
    handoff (chains finished on host threads from the GPU's midstate, the GPU's prefix bytes)."""
    c, b = C.c_uint64(0), C.c_uint64(0)
    check(lib.krk_sha_last_tail(C.byref(c), C.byref(b)))
    return {"chains": c.value, "gpu_prefix_bytes": b.value}


def sha_offload_plan(lengths, threads: int, cus: int = 0, mode: int = OFFLOAD_DEVICE):
    """krk_host_offload_plan: (indices of the blobs the host would take, longest first,
    modelled GPU seconds, modelled host seconds) -- no device work (planner_rates(); cus
    > 0 overrides their CU count).  mode: a batch in
    HBM (OFFLOAD_DEVICE), host blobs hashed only (OFFLOAD_HOST_SHA, sha256_host) or hashed
    and piece-summed on the host (OFFLOAD_HOST_WHOLE, metainfo_digest_host)."""
    L = np.ascontiguousarray(lengths, dtype=np.uint64)
    idx = np.zeros(max(L.size, 1), dtype=np.uint32)
    k, g, h = C.c_uint64(0), C.c_double(0), C.c_double(0)
    check(lib.krk_host_offload_plan(L.ctypes.data_as(C.POINTER(C.c_uint64)), L.size, int(threads), int(cus),
                                    int(mode), idx.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(k), C.byref(g),
                                    C.byref(h)))
    return idx[:k.value].copy(), g.value, h.value


def set_devices(devs):
    """The process's device set (krk_set_devices): where the *_multi calls run and new
    Digesters / piece streams are placed; repeats allowed; [] = the calling thread's device."""
    arr = (C.c_int * max(len(devs), 1))(*devs)
    check(lib.krk_set_devices(arr, len(devs)))


def get_devices():
    n = C.c_uint32()
    check(lib.krk_get_devices(None, 0, C.byref(n)))
    arr = (C.c_int * max(n.value, 1))()
    check(lib.krk_get_devices(arr, n.value, C.byref(n)))
    return list(arr[:n.value])


def metainfo_digest_host(datas, piece_lengths, multi: bool = False):
    """End-to-end batch over HOST buffers (numpy uint8 arrays, pageable or
    pinned): one PCIe pass feeds both kernels.  Returns (sums per blob, digests).
    multi: krk_metainfo_digest_host_multi (LPT over the device set)."""
    n = len(datas)
    pls = np.broadcast_to(np.asarray(piece_lengths, dtype=np.int64), (n,))
    counts = [int(lib.krk_num_pieces(int(d.size), int(p))) for d, p in zip(datas, pls)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(counts) if n else []
    arr = (krk_blob * max(n, 1))()
    for i, d in enumerate(datas):
        arr[i] = krk_blob(d.ctypes.data if d.size else None, int(d.size), int(pls[i]), int(offs[i]))
    sums = np.zeros(max(int(offs[-1]), 1), dtype=np.uint32)
    dg = np.zeros((max(n, 1), 32), dtype=np.uint8)
    fn = lib.krk_metainfo_digest_host_multi if multi else lib.krk_metainfo_digest_host
    check(fn(arr, n, sums.ctypes.data_as(C.POINTER(C.c_uint32)), dg.ctypes.data_as(C.POINTER(C.c_uint8))))
    return [sums[int(offs[i]):int(offs[i + 1])] for i in range(n)], dg[:n]


def metainfo_digest_files(paths, lengths, piece_lengths, multi: bool = False):
    """krk_metainfo_digest_files: the digests and piece sums of CAS files, each read once
    (pinned windows -> both kernels; the planner's files on host threads).  lengths: the
    sizes the caller stat-ed.  Returns (sums per file, digests).  multi: the _multi form
    (LPT over the device set)."""
    n = len(paths)
    L = np.asarray(lengths, dtype=np.uint64)
    pls = np.broadcast_to(np.asarray(piece_lengths, dtype=np.int64), (n,))
    counts = [int(lib.krk_num_pieces(int(l), int(p))) for l, p in zip(L, pls)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(counts) if n else []
    enc = [p.encode() if isinstance(p, str) else bytes(p) for p in paths]
    arr = (krk_file_blob * max(n, 1))()
    for i in range(n):
        arr[i] = krk_file_blob(enc[i], int(L[i]), int(pls[i]), int(offs[i]))
    sums = np.zeros(max(int(offs[-1]), 1), dtype=np.uint32)
    dg = np.zeros((max(n, 1), 32), dtype=np.uint8)
    fn = lib.krk_metainfo_digest_files_multi if multi else lib.krk_metainfo_digest_files
    check(fn(arr, n, sums.ctypes.data_as(C.POINTER(C.c_uint32)), dg.ctypes.data_as(C.POINTER(C.c_uint8))))
    return [sums[int(offs[i]):int(offs[i + 1])] for i in range(n)], dg[:n]


def piece_sums_files(paths, lengths, piece_lengths, multi: bool = False):
    """krk_piece_sums_files: the piece sums of CAS files (Generate over cache files), on the
    CRC placement (krk_set_crc_placement; AUTO = the measured crossover).  Returns the sums
    per file as one array (offsets from the counts) and the per-file views."""
    n = len(paths)
    L = np.asarray(lengths, dtype=np.uint64)
    pls = np.broadcast_to(np.asarray(piece_lengths, dtype=np.int64), (n,))
    counts = [int(lib.krk_num_pieces(int(l), int(p))) for l, p in zip(L, pls)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(counts) if n else []
    enc = [p.encode() if isinstance(p, str) else bytes(p) for p in paths]
    arr = (krk_file_blob * max(n, 1))()
    for i in range(n):
        arr[i] = krk_file_blob(enc[i], int(L[i]), int(pls[i]), int(offs[i]))
    sums = np.zeros(max(int(offs[-1]), 1), dtype=np.uint32)
    fn = lib.krk_piece_sums_files_multi if multi else lib.krk_piece_sums_files
    check(fn(arr, n, sums.ctypes.data_as(C.POINTER(C.c_uint32))))
    return sums, offs


PLACE_AUTO, PLACE_HOST, PLACE_GPU = 0, 1, 2


def set_crc_placement(placement: int):
    """krk_set_crc_placement: the process-wide placement of CRC-only host calls."""
    check(lib.krk_set_crc_placement(int(placement)))


def windows_last_call() -> dict:
    """The calling thread's last krk_metainfo_digest_host / _files call: the most live blobs
    in a window, the windows, the blobs the host offload took (krk_windows_last_call)."""
    m, w, h, d = C.c_uint64(), C.c_int(), C.c_uint64(), C.c_int()
    g, rb, rs = C.c_int(), C.c_uint64(), C.c_double()
    check(lib.krk_windows_last_call(C.byref(m), C.byref(w), C.byref(h)))
    check(lib.krk_windows_last_direct(C.byref(d)))
    check(lib.krk_windows_last_gather(C.byref(g), C.byref(rb), C.byref(rs)))
    ph = [C.c_double() for _ in range(5)]
    dr = C.c_int()
    check(lib.krk_windows_last_phases(*[C.byref(x) for x in ph], C.byref(dr)))
    lc = C.c_uint64()
    check(lib.krk_windows_last_copyout(C.byref(lc)))
    return {"live_registered_at_copyout": lc.value, "max_live": m.value, "windows": w.value, "host_blobs": h.value, "direct_windows": d.value,
            "gather_windows": g.value, "registered_bytes": rb.value, "register_s": rs.value,
            "phases_s": dict(zip(("loop", "acquire", "fill", "enqueue"), (round(x.value, 4) for x in ph[:4]))),
            "resident_sample": round(ph[4].value, 4), "direct_reads": bool(dr.value)}


def set_host_gather(mode: int):
    """krk_set_host_gather: -1 AUTO (default), 0 stage every window, 1 gather any size."""
    check(lib.krk_set_host_gather(int(mode)))


def device_pci_bus_id() -> str:
    b = C.create_string_buffer(64)
    check(lib.krk_device_pci_bus_id(b, 64))
    return b.value.decode()


def device_cus() -> int:
    v = C.c_int(0)
    check(lib.krk_device_cus(C.byref(v)))
    return v.value


def window_stream_cap() -> int:
    v = C.c_uint64(0)
    check(lib.krk_window_stream_cap(C.byref(v)))
    return v.value


class ChunkedBatch:
    """Window-by-window metainfo+digest over device chunks (krk_metainfo_digest_chunks_dev):
    per-blob SHA midstates and XOR-accumulated piece sums live on the device between steps."""

    def __init__(self, lengths, piece_lengths):
        self.lengths = np.asarray(lengths, dtype=np.uint64)
        n = len(self.lengths)
        self.piece_lengths = np.array(np.broadcast_to(np.asarray(piece_lengths, dtype=np.int64), (n,)))
        self.n_pieces = np.array([lib.krk_num_pieces(int(L), int(p)) for L, p in
                                  zip(self.lengths, self.piece_lengths)], dtype=np.uint64)
        self.sums_off = np.zeros(n, dtype=np.uint64)
        if n:
            self.sums_off[1:] = np.cumsum(self.n_pieces)[:-1]
        self.total_pieces = int(self.n_pieces.sum())
        self.state = DeviceBuffer(max(n, 1) * 32)
        self.sums = DeviceBuffer(max(self.total_pieces, 1) * 4)
        self.sums.zero()
        self.digests = DeviceBuffer(max(n, 1) * 32)

    def step_arrays(self, blob_idx, ptrs, offsets, lengths, stream=None, sha_stream=None, crc_after_sha=False):
        """step() from numpy arrays (one window of thousands of chunks, no Python loop);
        sha_stream: the SHA-256 launch's stream (krk_metainfo_digest_chunks_dev_on);
        crc_after_sha: the CRCs on `stream` once that launch has ended (_after)."""
        arr = chunk_array(ptrs, offsets, lengths, self.lengths[blob_idx], self.piece_lengths[blob_idx],
                          self.sums_off[blob_idx], blob_idx)
        fn = lib.krk_metainfo_digest_chunks_dev_after if crc_after_sha else lib.krk_metainfo_digest_chunks_dev_on
        check(fn(arr.ctypes.data_as(C.POINTER(krk_chunk)), len(arr), self.state.ptr, self.sums.ptr, self.digests.ptr,
                 stream, sha_stream))

    def step(self, items, stream=None):
        """items: [(blob index, device address of the chunk, offset, length)]."""
        arr = (krk_chunk * max(len(items), 1))()
        for k, (i, ptr, off, ln) in enumerate(items):
            arr[k] = krk_chunk(ptr, int(off), int(ln), int(self.lengths[i]), int(self.piece_lengths[i]),
                               int(self.sums_off[i]), int(i))
        check(lib.krk_metainfo_digest_chunks_dev(arr, len(items), self.state.ptr, self.sums.ptr,
                                                 self.digests.ptr, stream))


KRK_CHUNK_DTYPE = np.dtype([("data", "<u8"), ("offset", "<u8"), ("length", "<u8"), ("blob_length", "<u8"),
                            ("piece_length", "<i8"), ("sums_offset", "<u8"), ("blob", "<u8")])
assert KRK_CHUNK_DTYPE.itemsize == C.sizeof(krk_chunk)


def chunk_array(ptrs, offsets, lengths, blob_lengths, piece_lengths, sums_offsets, blobs) -> np.ndarray:
    """A krk_chunk[] built column-wise with numpy."""
    n = len(ptrs)
    arr = np.zeros(max(n, 1), dtype=KRK_CHUNK_DTYPE)[:n]
    arr["data"], arr["offset"], arr["length"] = ptrs, offsets, lengths
    arr["blob_length"], arr["piece_length"] = blob_lengths, piece_lengths
    arr["sums_offset"], arr["blob"] = sums_offsets, blobs
    return arr


def synth_fill_chunk_arrays(blob_ids, ptrs, offsets, lengths, variant: int = 0, stream=None):
    """synth_fill_chunks from numpy arrays."""
    n = len(ptrs)
    arr = chunk_array(ptrs, offsets, lengths, 0, 1, 0, blob_ids)
    check(lib.krk_synth_fill_chunks_dev(arr.ctypes.data_as(C.POINTER(krk_chunk)), n, variant, stream))


def synth_fill_chunks(items, variant: int = 0, stream=None):
    """items: [(blob id, device address, offset, length)] -> bytes [offset, offset+length)
    of each synthetic blob written at its address, one launch."""
    arr = (krk_chunk * max(len(items), 1))()
    for k, (b, ptr, off, ln) in enumerate(items):
        arr[k] = krk_chunk(ptr, int(off), int(ln), 0, 1, 0, int(b))
    check(lib.krk_synth_fill_chunks_dev(arr, len(items), variant, stream))


_NODES_CACHE: dict = {}


def nodes_struct(labels, weights):
    """krk_nodes for (labels, weights), kept per membership (the last 16) so a placement
    call per batch does not re-encode the ring."""
    key = (tuple(labels), tuple(int(w) for w in weights))
    hit = _NODES_CACHE.get(key)
    if hit is not None:
        return hit
    if len(_NODES_CACHE) >= 16:
        _NODES_CACHE.pop(next(iter(_NODES_CACHE)))
    _NODES_CACHE[key] = hit = _nodes_struct(labels, weights)
    return hit


def _nodes_struct(labels, weights):
    enc = [s.encode() for s in labels]
    blob = b"".join(enc)
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(e) for e in enc])
    w = np.ascontiguousarray(weights, dtype=np.int64)
    s = krk_nodes(blob, off.ctypes.data_as(C.POINTER(C.c_uint64)), w.ctypes.data_as(C.POINTER(C.c_int64)),
                  len(labels))
    return s, (blob, off, w)  # keep the backing arrays alive


def ring_locations_dev(digests_dev: DeviceBuffer, n: int, labels, healthy, max_replica: int,
                       locs_dev: DeviceBuffer, counts_dev: DeviceBuffer, stream=None, weights=None):
    """ring.Locations for n device-resident digests; weights default to the ring's 100
    (lib/hashring/ring.go:28)."""
    s, keep = nodes_struct(labels, [100] * len(labels) if weights is None else weights)
    h = np.ascontiguousarray(healthy, dtype=np.uint8)
    check(lib.krk_ring_locations_dev(digests_dev.ptr, n, C.byref(s), h.ctypes.data_as(C.POINTER(C.c_uint8)),
                                      max_replica, locs_dev.ptr, counts_dev.ptr, stream))
    del keep


def ring_locations_u8_dev(digests_dev: DeviceBuffer, n: int, labels, healthy, max_replica: int,
                          locs_dev: DeviceBuffer, counts_dev: DeviceBuffer, stream=None, weights=None):
    """ring_locations_dev with uint8 owner indices (0xFF padded) for rings of <= 255 nodes:
    a quarter of the owner-list bytes to copy back (krk_ring_locations_u8_dev)."""
    s, keep = nodes_struct(labels, [100] * len(labels) if weights is None else weights)
    h = np.ascontiguousarray(healthy, dtype=np.uint8)
    check(lib.krk_ring_locations_u8_dev(digests_dev.ptr, n, C.byref(s), h.ctypes.data_as(C.POINTER(C.c_uint8)),
                                         max_replica, locs_dev.ptr, counts_dev.ptr, stream))
    del keep


class KernelTimer:
    """hipEvent-based per-kernel device time (recorded on each kernel's stream)."""

    def __enter__(self):
        check(lib.krk_set_timing(1))
        check(lib.krk_reset_kernel_stats())
        return self

    def __exit__(self, *a):
        check(lib.krk_set_timing(0))

    @staticmethod
    def timeline(kernel: str):
        """[(plan, units, start_ms, end_ms)] of every timed launch of `kernel` since the
        timer was entered (krk_kernel_timeline)."""
        n = C.c_uint64()
        check(lib.krk_kernel_timeline(kernel.encode(), None, 0, C.byref(n)))
        recs = (krk_launch_rec * max(1, n.value))()
        check(lib.krk_kernel_timeline(kernel.encode(), recs, n.value, C.byref(n)))
        return [(r.plan, r.units, r.start_ms, r.end_ms) for r in recs[:n.value]]

    @staticmethod
    def stats(kernel: str):
        n = C.c_uint64()
        ms = C.c_double()
        check(lib.krk_kernel_stats(kernel.encode(), C.byref(n), C.byref(ms)))
        return n.value, ms.value
