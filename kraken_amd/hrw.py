"""Host-side mirror of lib/hrw (weighted rendezvous hashing) over the C ABI.

Mirrors lib/hrw/rendezvous.go: ``Murmur3Hash`` (:39) + ``UInt64ToFloat64``
(:99-118) scoring, ``RendezvousHash.AddNode/RemoveNode/GetNode`` (:175-202) and
``GetOrderedNodes`` (:207-217).  Scores are computed on the GPU
(hrw_place.hip); exact score ties go to the lower node index (the reference's
tie order follows Go map iteration, lib/hashring/ring.go:151, i.e. unspecified).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import KRK_EHEX, KrakenError, check, krk_nodes, lib


class RendezvousHashNode:
    __slots__ = ("RHash", "Label", "Weight")

    def __init__(self, rhash: "RendezvousHash", label: str, weight: int):
        self.RHash, self.Label, self.Weight = rhash, label, int(weight)

    def Score(self, key: str) -> float:
        """RendezvousHashNode.Score (rendezvous.go:151-172); NaN for invalid hex."""
        nodes = [self]
        _, scores = _ordered([key], nodes, 1, want_scores=True)
        return float(scores[0, 0])

    def __repr__(self):
        return f"RendezvousHashNode({self.Label!r}, {self.Weight})"


class _NodeTable:
    """krk_nodes view kept alive with its backing arrays."""

    def __init__(self, nodes):
        enc = [n.Label.encode() for n in nodes]
        self.blob = b"".join(enc)
        self.off = np.zeros(len(enc) + 1, dtype=np.uint64)
        if enc:
            self.off[1:] = np.cumsum([len(e) for e in enc])
        self.w = np.ascontiguousarray([n.Weight for n in nodes], dtype=np.int64)
        self.s = krk_nodes(self.blob, self.off.ctypes.data_as(C.POINTER(C.c_uint64)),
                           self.w.ctypes.data_as(C.POINTER(C.c_int64)), len(nodes))


def _ordered(keys, nodes, n_out: int, want_scores: bool = False):
    kb = [k.encode() for k in keys]
    blob = b"".join(kb)
    off = np.zeros(len(kb) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(k) for k in kb])
    nt = _NodeTable(nodes)
    order = np.full((len(keys), max(n_out, 1)), -1, dtype=np.int32)
    scores = np.zeros((len(keys), len(nodes)), dtype=np.float64) if want_scores else None
    rc = lib.krk_hrw_ordered(blob, off.ctypes.data_as(C.POINTER(C.c_uint64)), len(keys), C.byref(nt.s),
                             n_out, order.ctypes.data_as(C.POINTER(C.c_int32)),
                             scores.ctypes.data_as(C.POINTER(C.c_double)) if want_scores else None)
    if rc not in (0, KRK_EHEX):
        check(rc)
    return order[:, :n_out], scores


def _check_n(n: int) -> None:
    # The reference slices nodes[:n] (rendezvous.go:216), which panics for n < 0.
    if n < 0:
        raise ValueError(f"slice bounds out of range [:{n}]")


class RendezvousHash:
    """lib/hrw/rendezvous.go:55-60.  Hash is always murmur3 (ring.go:150); the
    reference's other HashFactory/ScoreFunc choices are test-only."""

    def __init__(self):
        self.Nodes: list[RendezvousHashNode] = []

    def AddNode(self, seed: str, weight: int) -> None:
        self.Nodes.append(RendezvousHashNode(self, seed, weight))

    def RemoveNode(self, name: str) -> None:
        for i, n in enumerate(self.Nodes):
            if n.Label == name:
                del self.Nodes[i]
                break

    def GetNode(self, name: str):
        for i, n in enumerate(self.Nodes):
            if n.Label == name:
                return n, i
        return None, -1

    def GetOrderedNodes(self, key: str, n: int) -> list[RendezvousHashNode]:
        _check_n(n)
        if not self.Nodes:
            return []
        m = min(n, len(self.Nodes))
        order, _ = _ordered([key], self.Nodes, m)
        return [self.Nodes[int(j)] for j in order[0, :m]]

    def GetOrderedNodesBatch(self, keys, n: int) -> np.ndarray:
        """Batched GetOrderedNodes: int32 [len(keys), min(n, N)] node indices."""
        _check_n(n)
        m = min(n, len(self.Nodes))
        order, _ = _ordered(list(keys), self.Nodes, m)
        return order

    def Scores(self, keys) -> np.ndarray:
        """float64 [len(keys), N]: Score of every node for every key."""
        _, s = _ordered(list(keys), self.Nodes, len(self.Nodes), want_scores=True)
        return s


def NewRendezvousHash() -> RendezvousHash:
    return RendezvousHash()


def UInt64ToFloat64(bytes_uint: bytes, max_value: bytes = b"\xff" * 8, rehash=None) -> float:
    """rendezvous.go:99-118 on the host (the device path computes the same in
    hrw_place.hip): the low 53 bits of the big-endian value, re-hashed once by
    `rehash(bytes) -> 8 bytes` when they are all zero, divided by 2^53."""
    ones53 = int.from_bytes(max_value[:8], "big") >> 11
    val = int.from_bytes(bytes_uint[:8], "big") & ones53
    if val == 0 and rehash is not None:
        val = int.from_bytes(rehash(bytes_uint)[:8], "big") & ones53
    return float(val) / float(1 << 53)


def _round_prec(v: int, prec: int) -> int:
    """Round a non-negative integer to `prec` significant bits, ties to even
    (big.Float.SetPrec's default rounding mode)."""
    extra = v.bit_length() - prec
    if extra <= 0:
        return v
    q, r = divmod(v, 1 << extra)
    half = 1 << (extra - 1)
    if r > half or (r == half and q & 1):
        q += 1
    return q << extra


def BigIntToFloat64(bytes_uint: bytes, max_value: bytes, hasher=None) -> float:
    """rendezvous.go:120-146 (test-only in the reference; no ring uses it):
    big.Float(hash) rounded to 53 bits, divided by big.Float(max) into a
    53-bit result (round to nearest even), returned as float64."""
    del hasher  # unused by the reference too
    h = _round_prec(int.from_bytes(bytes_uint, "big"), 53)
    m = int.from_bytes(max_value, "big")
    if m == 0:
        raise ZeroDivisionError("BigIntToFloat64: zero max value")
    # Python's int / int true division is correctly rounded to the nearest double
    # (53-bit significand, ties to even) -- big.Float.Quo at prec 53 + Float64().
    return h / m


__all__ = ["RendezvousHash", "RendezvousHashNode", "NewRendezvousHash", "UInt64ToFloat64", "BigIntToFloat64",
           "KrakenError"]
