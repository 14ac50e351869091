"""Weighted rendezvous placement of the CAS store's 256 shard directories over
volumes (lib/store/ca_store.go:137-171, initCASVolumes): for subdir "%02X" the
top node of GetOrderedNodes(subdir, 1) over the volumes (murmur3 +
UInt64ToFloat64, per-volume weights) owns it; the store symlinks
<dir>/<subdir> -> <volume>/<basename(dir)>/<subdir>.  The ordering runs on the
GPU through the same HRW kernel as the hashring (krk_hrw_ordered)."""
from __future__ import annotations

import os
import posixpath

from .hrw import NewRendezvousHash


class Volume:
    def __init__(self, Location: str, Weight: int):
        self.Location, self.Weight = Location, int(Weight)


def volume_subdirs(volumes) -> dict:
    """{subdir "%02X": volume location} for the 256 shard directories."""
    rh = NewRendezvousHash()
    for v in volumes:
        rh.AddNode(v.Location, v.Weight)
    keys = [f"{i:02X}" for i in range(256)]
    order = rh.GetOrderedNodesBatch(keys, 1)
    return {k: rh.Nodes[int(order[i, 0])].Label for i, k in enumerate(keys)}


def initCASVolumes(dir_: str, volumes) -> None:
    """ca_store.go:137-171 with the same error strings."""
    if not volumes:
        return
    for v in volumes:
        if not os.path.exists(v.Location):
            raise OSError(f"verify volume: stat {v.Location}: no such file or directory")
    base = posixpath.basename(posixpath.normpath(dir_)) if dir_ else "."  # Go path.Base
    for sub, loc in volume_subdirs(volumes).items():
        src = posixpath.join(loc, base, sub)
        try:
            os.makedirs(src, mode=0o775, exist_ok=True)
        except OSError as e:
            raise OSError(f"volume source path: {e}") from e
        tgt = posixpath.join(dir_, sub)
        try:
            _create_or_update_symlink(src, tgt)
        except OSError as e:
            raise OSError(f"symlink to volume: {e}") from e


def _create_or_update_symlink(src: str, tgt: str) -> None:
    """createOrUpdateSymlink (lib/store/utils.go:25-47): an existing target that is not
    a symlink (a regular file, a real directory) is an error and is left in place;
    a symlink to another source is replaced; a missing target is created."""
    try:
        os.stat(tgt)  # follows links, like os.Stat
    except FileNotFoundError:
        os.symlink(src, tgt)
        return
    existing = os.readlink(tgt)  # OSError (EINVAL) when tgt is not a symlink
    if existing != src:
        os.remove(tgt)
        os.symlink(src, tgt)
