"""Host-side mirror of lib/hashring's owner-list computation over the C ABI.

``Ring.Locations`` follows lib/hashring/ring.go:91-118: the HRW order of the
digest's ShardID (core/digest.go:148-150) over every member (weight 100,
ring.go:28,150-153), then the healthy filter: no healthy node -> [order[0]];
else walk the order while (no location yet or i < MaxReplica), keeping healthy
nodes.  Membership/health monitoring (Monitor/Refresh) is out of scope: the
caller passes the member list and the healthy set.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, lib
from .hrw import _NodeTable, RendezvousHash

DEFAULT_WEIGHT = 100  # ring.go:28
DEFAULT_MAX_REPLICA = 3  # lib/hashring/config.go:30-37


class Ring:
    def __init__(self, addrs, healthy=None, max_replica: int = DEFAULT_MAX_REPLICA):
        self.addrs = list(addrs)
        if not self.addrs:
            raise ValueError("ring must be non-empty")
        self.hash = RendezvousHash()
        for a in self.addrs:
            self.hash.AddNode(a, DEFAULT_WEIGHT)
        self.max_replica = int(max_replica)
        self.set_healthy(self.addrs if healthy is None else healthy)

    def set_healthy(self, healthy) -> None:
        hs = set(healthy)
        self._healthy = np.array([1 if a in hs else 0 for a in self.addrs], dtype=np.uint8)

    def Contains(self, addr: str) -> bool:
        return addr in self.addrs

    def _raw(self, digests32: np.ndarray):
        d = np.ascontiguousarray(digests32, dtype=np.uint8).reshape(-1, 32)
        n = d.shape[0]
        row = max(1, self.max_replica)
        locs = np.full((n, row), -1, dtype=np.int32)
        counts = np.zeros(n, dtype=np.uint8)
        nt = _NodeTable(self.hash.Nodes)
        check(lib.krk_ring_locations(d.ctypes.data_as(C.POINTER(C.c_uint8)), n, C.byref(nt.s),
                                     self._healthy.ctypes.data_as(C.POINTER(C.c_uint8)), self.max_replica,
                                     locs.ctypes.data_as(C.POINTER(C.c_int32)),
                                     counts.ctypes.data_as(C.POINTER(C.c_uint8))))
        return locs, counts

    def Locations(self, d) -> list[str]:
        raw = np.frombuffer(bytes.fromhex(d.Hex()), dtype=np.uint8)
        locs, counts = self._raw(raw)
        return [self.addrs[int(j)] for j in locs[0, : counts[0]]]

    def LocationsBatch(self, digests32: np.ndarray):
        """Raw 32-byte digests -> (int32 [n, max(1,MaxReplica)] node indices, uint8 [n] counts)."""
        return self._raw(digests32)
