"""error paths.

* A HIP error left pending on a thread by an earlier call that nobody checked is reported
  by the next launch of the library, under that entry point, as coming from the earlier
  call -- not cleared away -- and the thread is clean afterwards.
* An error the library itself reports (here an impossible allocation) is consumed when it
  is reported: it does not resurface in the next call's launch.
* The engine's caller-runs dispatch launches on the engine's device from the caller's
  thread and leaves the caller's current device as it was."""
import ctypes as C

import numpy as np
import pytest

from kraken_amd import device as D
from kraken_amd._capi import KRK_EHIP, KRK_ENOMEM, KRK_PLACE_GPU, check, lib

pytestmark = pytest.mark.gpu


def _hip():
    """The HIP runtime the library itself is linked against (already loaded)."""
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line and "/opt/rocm" in line:
            return C.CDLL(line.split()[-1])
    return C.CDLL("/opt/rocm/lib/libamdhip64.so")


def test_pending_error_is_reported_by_the_next_launch(gpu, orc):
    hip = _hip()
    arena = D.BlobArena([3 << 20], 1 << 20, blob_ids=[3])
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)  # a clean launch first
    D.synchronize()
    assert hip.hipSetDevice(1 << 20) != 0  # an unchecked failure: hipErrorInvalidDevice left pending
    rc = lib.krk_piece_sums_dev(arena.blob_structs(), 1, out.sums.ptr, None)
    msg = lib.krk_last_error().decode()
    assert rc == KRK_EHIP, (rc, msg)
    assert "crc32_pieces launch" in msg and "pending from an earlier call" in msg, msg
    assert hip.hipGetLastError() == 0  # reported once, not left behind
    check(lib.krk_piece_sums_dev(arena.blob_structs(), 1, out.sums.ptr, None))
    D.synchronize()
    sums = out.sums.to_host(np.uint32, arena.total_pieces)
    ref = orc.calc_piece_sums(orc.synth(3, 3 << 20), 1 << 20)[1]
    assert np.array_equal(sums, ref)


def test_library_reported_error_does_not_resurface(gpu):
    p = C.c_void_p()
    assert lib.krk_dev_alloc(1 << 62, C.byref(p)) == KRK_ENOMEM
    assert "hipMalloc" in lib.krk_last_error().decode()
    arena = D.BlobArena([1000], 64, blob_ids=[1])
    out = D.BatchOutputs(arena)
    check(lib.krk_metainfo_digest_dev(arena.blob_structs(), 1, out.sums.ptr, out.digests.ptr, None))
    D.synchronize()


def test_caller_runs_dispatch_keeps_the_callers_device(gpu):
    """The digester's engine lives on device 0; a submission that completes the coalescing
    set launches the batch on the caller's thread (caller-runs dispatch) and must restore
    the thread's current device.  With one device, the check is that hipGetDevice still
    answers the device the thread selected and later launches on this thread work."""
    hip = _hip()
    h = C.c_void_p()
    check(lib.krk_digester_new_on(KRK_PLACE_GPU, C.byref(h)))
    try:
        data = np.arange(3 << 20, dtype=np.uint8)
        check(lib.krk_digester_write(h, data.ctypes.data, data.size))
        o = (C.c_uint8 * 32)()
        check(lib.krk_digester_sum(h, o))
        import hashlib
        assert bytes(o) == hashlib.sha256(data.tobytes()).digest()
    finally:
        lib.krk_digester_free(h)
    dev = C.c_int(-1)
    assert hip.hipGetDevice(C.byref(dev)) == 0 and dev.value == 0
