"""ctypes binding of libkraken_hip.so (include/kraken_hip.h, and the benchmark / test
hooks of include/kraken_hip_internal.h).

This is the Python-side FFI stub over the C ABI -- the same role the cgo stubs in
INTEGRATION.md play for the reference's Go code.  There is no fallback: if the
HIP library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KRK_LIB_PATH") or os.path.join(_HERE, "lib", "libkraken_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "kraken_hip.h")
INTERNAL_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "kraken_hip_internal.h")

KRK_OK, KRK_EINVAL, KRK_EHIP, KRK_ENOMEM, KRK_ENODEV, KRK_ERANGE, KRK_EHEX, KRK_EIO = 0, -1, -2, -3, -4, -5, -6, -7
KRK_PLACE_AUTO, KRK_PLACE_HOST, KRK_PLACE_GPU = 0, 1, 2
KRK_OFFLOAD_AUTO = -1


class KrakenError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class krk_blob(C.Structure):
    _fields_ = [("data", C.c_void_p), ("length", C.c_uint64), ("piece_length", C.c_int64),
                ("sums_offset", C.c_uint64)]


class krk_file_blob(C.Structure):
    _fields_ = [("path", C.c_char_p), ("length", C.c_uint64), ("piece_length", C.c_int64),
                ("sums_offset", C.c_uint64)]


class krk_chunk(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offset", C.c_uint64), ("length", C.c_uint64),
                ("blob_length", C.c_uint64), ("piece_length", C.c_int64), ("sums_offset", C.c_uint64),
                ("blob", C.c_uint64)]


class krk_launch_rec(C.Structure):
    _fields_ = [("device", C.c_int32), ("plan", C.c_int32), ("units", C.c_uint64), ("start_ms", C.c_double),
                ("end_ms", C.c_double)]


class krk_planner_rates(C.Structure):
    _fields_ = [("sha_stream_bps", C.c_double * 3), ("d2h_bps", C.c_double), ("h2d_bps", C.c_double),
                ("host_sha_bps", C.c_double), ("host_crc_bps", C.c_double), ("host_copy_bps", C.c_double),
                ("cus", C.c_int32),
                ("source", C.c_int32)]


class krk_nodes(C.Structure):
    _fields_ = [("labels", C.c_char_p), ("label_off", C.POINTER(C.c_uint64)),
                ("weights", C.POINTER(C.c_int64)), ("n_nodes", C.c_uint32)]


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    vp, u8p, u32p, u64p, i32p, i64p, f64p = (C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint64), C.POINTER(C.c_int32),
                                              C.POINTER(C.c_int64), C.POINTER(C.c_double))
    blobp, nodesp = C.POINTER(krk_blob), C.POINTER(krk_nodes)
    i = C.c_int
    sig = {
        "krk_version": (C.c_char_p, []),
        "krk_last_error": (C.c_char_p, []),
        "krk_device_count": (i, [C.POINTER(C.c_int)]),
        "krk_set_device": (i, [i]),
        "krk_init": (i, [C.c_uint64]),
        "krk_shutdown": (i, []),
        "krk_synchronize": (i, []),
        "krk_num_pieces": (C.c_uint64, [C.c_uint64, C.c_int64]),
        "krk_piece_sums_dev": (i, [blobp, C.c_uint64, vp, vp]),
        "krk_metainfo_batch_dev": (i, [blobp, C.c_uint64, C.c_char_p, u64p, vp, u32p, C.POINTER(C.c_uint8), vp]),
        "krk_piece_sums_host": (i, [blobp, C.c_uint64, u32p]),
        "krk_crc_host_split": (i, [u64p, u64p, f64p]),
        "krk_piece_sums_files": (i, [C.POINTER(krk_file_blob), C.c_uint64, u32p]),
        "krk_piece_stream_begin": (i, [C.c_int64, C.POINTER(vp)]),
        "krk_piece_stream_update": (i, [vp, vp, C.c_uint64]),
        "krk_piece_stream_end": (i, [vp, u32p, C.c_uint64, u64p, u64p]),
        "krk_piece_stream_free": (None, [vp]),
        "krk_crc32_update": (i, [C.c_uint32, vp, C.c_uint64, u32p]),
        "krk_crc32_update_on": (i, [i, C.c_uint32, vp, C.c_uint64, u32p]),
        "krk_set_crc_placement": (i, [i]),
        "krk_piece_stream_begin_on": (i, [i, C.c_int64, C.POINTER(vp)]),
        "krk_piece_stream_placement": (i, [vp, C.POINTER(C.c_int)]),
        "krk_verify_pieces_dev": (i, [blobp, u32p, u8p, vp]),
        "krk_verify_pieces_host": (i, [C.POINTER(vp), u64p, u32p, C.c_uint64, u8p]),
        "krk_sha256_dev": (i, [C.POINTER(vp), u64p, C.c_uint64, vp, vp]),
        "krk_sha256_host": (i, [C.POINTER(vp), u64p, C.c_uint64, u8p]),
        "krk_sha256_dev_on_host": (i, [C.POINTER(vp), u64p, C.c_uint64, i, vp, u8p]),
        "krk_digester_new": (i, [C.POINTER(vp)]),
        "krk_digester_new_on": (i, [i, C.POINTER(vp)]),
        "krk_digester_placement": (i, [vp, C.POINTER(C.c_int)]),
        "krk_set_digester_host_streams": (i, [C.c_int64]),
        "krk_engine_stats": (i, [u64p, u64p, u64p, u64p, u64p]),
        "krk_engine_set_pool_cap": (i, [C.c_uint64, u64p, u64p]),
        "krk_planner_rates_get": (i, [C.POINTER(krk_planner_rates)]),
        "krk_planner_rates_set": (i, [C.POINTER(krk_planner_rates)]),
        "krk_set_devices": (i, [C.POINTER(C.c_int), C.c_uint32]),
        "krk_get_devices": (i, [C.POINTER(C.c_int), C.c_uint32, C.POINTER(C.c_uint32)]),
        "krk_metainfo_digest_host_multi": (i, [blobp, C.c_uint64, u32p, u8p]),
        "krk_piece_sums_host_multi": (i, [blobp, C.c_uint64, u32p]),
        "krk_piece_sums_files_multi": (i, [C.POINTER(krk_file_blob), C.c_uint64, u32p]),
        "krk_sha256_host_multi": (i, [C.POINTER(vp), u64p, C.c_uint64, u8p]),
        "krk_host_sha256": (i, [vp, C.c_uint64, u8p]),
        "krk_host_crc32_update": (i, [C.c_uint32, vp, C.c_uint64, u32p]),
        "krk_hrw_uint64_to_float64": (i, [u8p, C.c_uint64, i, f64p]),
        "krk_set_sha_plan": (i, [i]),
        "krk_device_clock_mhz": (i, [vp, f64p]),
        "krk_digester_write": (i, [vp, vp, C.c_uint64]),
        "krk_digester_sum": (i, [vp, u8p]),
        "krk_digester_free": (None, [vp]),
        "krk_metainfo_digest_dev": (i, [blobp, C.c_uint64, vp, vp, vp]),
        "krk_metainfo_digest_host": (i, [blobp, C.c_uint64, u32p, u8p]),
        "krk_metainfo_digest_files": (i, [C.POINTER(krk_file_blob), C.c_uint64, u32p, u8p]),
        "krk_metainfo_digest_files_multi": (i, [C.POINTER(krk_file_blob), C.c_uint64, u32p, u8p]),
        "krk_window_sched_new": (i, [u64p, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(vp)]),
        "krk_window_sched_next": (i, [vp, u32p, u64p, u64p, C.c_uint64, u64p]),
        "krk_window_sched_free": (None, [vp]),
        "krk_window_sched_drop": (i, [vp, C.c_uint32, u64p]),
        "krk_window_sched_set_chunk_cap": (i, [vp, C.c_uint64]),
        "krk_chunks_crc_dev": (i, [C.POINTER(krk_chunk), C.c_uint64, vp, vp]),
        "krk_sha256_resume_dev_on_host": (i, [u32p, C.c_uint64, vp, C.c_uint64, i, u8p, vp]),
        "krk_sha256_resume_host": (i, [u32p, C.c_uint64, vp, C.c_uint64, i, u8p]),
        "krk_window_stream_cap": (i, [u64p]),
        "krk_windows_last_call": (i, [u64p, C.POINTER(C.c_int), u64p]),
        "krk_windows_last_direct": (i, [C.POINTER(C.c_int)]),
        "krk_windows_last_copyout": (i, [u64p]),
        "krk_windows_last_gather": (i, [C.POINTER(C.c_int), u64p, f64p]),
        "krk_windows_last_phases": (i, [f64p, f64p, f64p, f64p, f64p, C.POINTER(C.c_int)]),
        "krk_sha_last_tail": (i, [u64p, u64p]),
        "krk_sha_tail_plan": (i, [u64p, C.c_uint64, i, C.POINTER(C.c_uint32), u64p, u64p, f64p, f64p]),
        "krk_set_host_gather": (i, [i]),
        "krk_metainfo_digest_chunks_dev": (i, [C.POINTER(krk_chunk), C.c_uint64, vp, vp, vp, vp]),
        "krk_metainfo_digest_chunks_dev_on": (i, [C.POINTER(krk_chunk), C.c_uint64, vp, vp, vp, vp, vp]),
        "krk_metainfo_digest_chunks_dev_after": (i, [C.POINTER(krk_chunk), C.c_uint64, vp, vp, vp, vp, vp]),
        "krk_info_hash": (i, [C.c_int64, u32p, C.c_uint64, C.c_char_p, C.c_uint64, C.c_int64, u8p]),
        "krk_info_hash_batch": (i, [C.POINTER(C.c_int64), u32p, u64p, u64p, C.c_char_p, u64p, C.POINTER(C.c_int64),
                                    C.c_uint64, u8p]),
        "krk_bencode_info": (i, [C.c_int64, u32p, C.c_uint64, C.c_char_p, C.c_uint64, C.c_int64, u8p,
                                 C.c_uint64, u64p]),
        "krk_piece_length_for_size": (C.c_int64, [i64p, i64p, C.c_uint32, C.c_int64]),
        "krk_hrw_ordered": (i, [C.c_char_p, u64p, C.c_uint64, nodesp, C.c_uint32, i32p, f64p]),
        "krk_ring_locations": (i, [u8p, C.c_uint64, nodesp, u8p, C.c_int32, i32p, u8p]),
        "krk_ring_locations_dev": (i, [vp, C.c_uint64, nodesp, u8p, C.c_int32, vp, vp, vp]),
        "krk_ring_owner_table": (i, [nodesp, u8p, C.c_int32, i32p, u8p]),
        "krk_ring_locations_u8_dev": (i, [vp, C.c_uint64, nodesp, u8p, C.c_int32, vp, vp, vp]),
        "krk_synth_fill_dev": (i, [vp, C.c_uint64, C.c_uint64, C.c_uint64, i, vp]),
        "krk_synth_fill_chunks_dev": (i, [C.POINTER(krk_chunk), C.c_uint64, i, vp]),
        "krk_dev_alloc": (i, [C.c_uint64, C.POINTER(vp)]),
        "krk_dev_free": (i, [vp]),
        "krk_host_alloc": (i, [C.c_uint64, C.POINTER(vp)]),
        "krk_host_alloc_dma": (i, [C.c_uint64, C.POINTER(vp)]),
        "krk_host_free": (i, [vp]),
        "krk_memcpy_h2d": (i, [vp, vp, C.c_uint64]),
        "krk_memcpy_d2h": (i, [vp, vp, C.c_uint64]),
        "krk_memcpy_d2h_async": (i, [vp, vp, C.c_uint64, vp]),
        "krk_stream_create": (i, [C.POINTER(vp)]),
        "krk_stream_create_prio": (i, [i, C.POINTER(vp)]),
        "krk_device_cus": (i, [C.POINTER(i)]),
        "krk_device_pci_bus_id": (i, [C.c_char_p, C.c_uint32]),
        "krk_stream_destroy": (i, [vp]),
        "krk_stream_sync": (i, [vp]),
        "krk_event_create": (i, [C.POINTER(vp)]),
        "krk_event_record": (i, [vp, vp]),
        "krk_stream_wait_event": (i, [vp, vp]),
        "krk_event_create_polling": (i, [C.POINTER(vp)]),
        "krk_event_query": (i, [vp, C.POINTER(C.c_int)]),
        "krk_sha256_resume_stats": (i, [f64p, f64p]),
        "krk_sha256_resume_stats2": (i, [f64p, f64p]),
        "krk_event_sync": (i, [vp]),
        "krk_event_destroy": (i, [vp]),
        "krk_set_sha_host_offload": (i, [i]),
        "krk_sha_host_offload": (i, [C.POINTER(C.c_int)]),
        "krk_planner_calibrate": (i, []),
        "krk_sha_offload_plan": (i, [C.POINTER(C.c_uint64), C.c_uint64, i, i, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "krk_host_offload_plan": (i, [C.POINTER(C.c_uint64), C.c_uint64, i, i, i, C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "krk_set_timing": (i, [i]),
        "krk_sha_lanes_per_stream": (i, [C.c_uint64, C.POINTER(C.c_int)]),
        "krk_kernel_stats": (i, [C.c_char_p, u64p, f64p]),
        "krk_reset_kernel_stats": (i, []),
        "krk_kernel_timeline": (i, [C.c_char_p, C.POINTER(krk_launch_rec), C.c_uint64, u64p]),
        "krk_sha_plan_for": (i, [C.c_uint64, C.POINTER(C.c_int)]),
        "krk_host_cpu_budget": (i, [C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_uint32]),
        "krk_digester_host_streams": (i, [i64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    lib._krk_sigs = sig  # for tests: the bound surface
    return lib


lib = _load()


def check(rc: int) -> int:
    if rc != KRK_OK:
        raise KrakenError(rc, lib.krk_last_error().decode(errors="replace"))
    return rc


def _declared(path) -> set[str]:
    import re
    src = open(path).read()
    return set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(krk_[a-z0-9_]+)\s*\(", src, re.M))


def public_symbols() -> list[str]:
    """The drop-in boundary: every krk_* function declared in include/kraken_hip.h."""
    return sorted(_declared(HEADER_PATH))


def internal_symbols() -> list[str]:
    """Benchmark / test / diagnostic hooks declared in include/kraken_hip_internal.h."""
    return sorted(_declared(INTERNAL_HEADER_PATH))


def declared_symbols() -> list[str]:
    """Every krk_* function either header declares."""
    return sorted(set(public_symbols()) | set(internal_symbols()))


def host_cpu_budget() -> tuple[int, int, str]:
    """(this process's host CPU budget, the node's CPUs, where the budget came from):
    krk_host_cpu_budget, no device needed."""
    cpus, node = C.c_int(), C.c_int()
    src = C.create_string_buffer(64)
    check(lib.krk_host_cpu_budget(C.byref(cpus), C.byref(node), src, 64))
    return cpus.value, node.value, src.value.decode()
