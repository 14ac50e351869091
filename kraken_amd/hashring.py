"""Host-side mirror of lib/hashring's owner-list computation over the C ABI.

``Ring.Locations`` follows lib/hashring/ring.go:91-118: the HRW order of the
digest's ShardID (core/digest.go:148-150) over every member (weight 100,
ring.go:28,150-153), then the healthy filter: no healthy node -> [order[0]];
else walk the order while (no location yet or i < MaxReplica), keeping healthy
nodes.  Membership/health monitoring (Monitor, the health filters) is out of scope:
the caller passes the member list and the healthy set.

Locations depends on the digest only through its 2-byte ShardID, so Refresh (the
reference rebuilds its hrw object there, ring.go:141-165) computes all 65,536 owner
lists on the GPU in one call (krk_ring_owner_table) and Locations is a host lookup
-- the binding INTEGRATION.md gives the Go ring.
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
        self._table = None  # rebuilt by the next Refresh / Locations

    def Refresh(self) -> None:
        """The 65,536-row owner table for the current members and healthy set."""
        row = max(1, self.max_replica)
        locs = np.full((65536, row), -1, dtype=np.int32)
        counts = np.zeros(65536, dtype=np.uint8)
        nt = _NodeTable(self.hash.Nodes)
        check(lib.krk_ring_owner_table(C.byref(nt.s), self._healthy.ctypes.data_as(C.POINTER(C.c_uint8)),
                                       self.max_replica, locs.ctypes.data_as(C.POINTER(C.c_int32)),
                                       counts.ctypes.data_as(C.POINTER(C.c_uint8))))
        self._table = (locs, counts)

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
        """ring.Locations (lib/hashring/ring.go:91-118): a lookup of the ShardID's row."""
        if self._table is None:
            self.Refresh()
        locs, counts = self._table
        shard = int(d.ShardID(), 16)
        return [self.addrs[int(j)] for j in locs[shard, : counts[shard]]]

    def LocationsBatch(self, digests32: np.ndarray):
        """Raw 32-byte digests -> (int32 [n, max(1,MaxReplica)] node indices, uint8 [n] counts)."""
        return self._raw(digests32)
