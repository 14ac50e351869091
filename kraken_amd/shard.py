"""Blob sharding across GPUs (one process per GPU).

The path partitions by blob: every blob's piece sums and digest are computed on
exactly one GPU, with no exchange step, so the only multi-GPU machinery is (a) a
balanced assignment of blobs to ranks -- greedy LPT on bytes -- and (b) a
host-side gather of the small per-blob results (<= a few KB per blob) to rank 0.
No RCCL collective is on the data path.
"""
from __future__ import annotations

import heapq

import numpy as np


def lpt_shard(lengths, world: int) -> list[list[int]]:
    """Longest-processing-time-first: blobs sorted by size descending, each to the
    currently lightest rank.  Returns the blob indices of every rank (each list in
    ascending index order)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    heap = [(0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for i in np.argsort(-lengths.astype(np.int64), kind="stable"):
        load, r = heapq.heappop(heap)
        out[r].append(int(i))
        heapq.heappush(heap, (load + int(lengths[i]), r))
    return [sorted(x) for x in out]


def shard_loads(lengths, shards) -> list[int]:
    lengths = np.asarray(lengths, dtype=np.uint64)
    return [int(lengths[s].sum()) if s else 0 for s in shards]


def gather_results(local: dict, dist=None, dst: int = 0):
    """Gather {blob_index: result} dicts from every rank to `dst` (host objects over
    the process group's control plane)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    world = dist.get_world_size()
    objs = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(local, objs, dst=dst)
    if dist.get_rank() != dst:
        return None
    merged = {}
    for o in objs:
        merged.update(o)
    return merged
