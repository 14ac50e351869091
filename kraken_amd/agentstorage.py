"""Host-side mirror of the agent's piece verification.

``Torrent.WritePiece`` follows lib/torrent/storage/agentstorage/torrent.go:174-220:
length check ("invalid piece length: expected %d, got %d"), ErrPieceComplete for a
piece already written, CRC-32 of the received bytes against
``MetaInfo.GetPieceSum(pi)`` ("invalid piece sum"), then the bytes go to the
download file at the piece's offset and the piece is marked complete.

``Torrent.WritePieces`` is the batched form the reference lacks: the dispatcher
(lib/torrent/scheduler/dispatch/dispatcher.go:531-560) hands over every piece
received since the last call, and one ``krk_verify_pieces_host`` call checks them
all on the GPU instead of one ``hash.Hash32`` per piece.  The download-file and
piece-status machinery around it (CADownloadStore, pieces.go metadata) is out of
scope; a plain file stands in for it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import core
from ._capi import check, lib


class ErrPieceComplete(Exception):
    """storage.ErrPieceComplete (lib/torrent/storage/torrent.go)."""

    def __str__(self):
        return "piece is already complete"


def verify_pieces(datas, expected) -> np.ndarray:
    """ok[i] = crc32(datas[i]) == expected[i], one GPU pass over host buffers."""
    n = len(datas)
    ok = np.zeros(max(n, 1), dtype=np.uint8)
    if not n:
        return ok[:0].astype(bool)
    arrs = [np.frombuffer(memoryview(d), dtype=np.uint8) for d in datas]
    ptrs = (C.c_void_p * n)(*[a.ctypes.data if a.size else None for a in arrs])
    lens = np.ascontiguousarray([a.size for a in arrs], dtype=np.uint64)
    exp = np.ascontiguousarray(expected, dtype=np.uint32)
    check(lib.krk_verify_pieces_host(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)),
                                     exp.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                                     ok.ctypes.data_as(C.POINTER(C.c_uint8))))
    return ok[:n].astype(bool)


class Torrent:
    """agentstorage.Torrent's write path over one download file."""

    def __init__(self, mi: core.MetaInfo, path: str):
        self.mi = mi
        self.path = path
        self.complete = np.zeros(mi.NumPieces(), dtype=bool)
        if not os.path.exists(path):
            with open(path, "wb") as f:
                f.truncate(mi.Length())

    def NumPieces(self) -> int:
        return self.mi.NumPieces()

    def PieceLength(self, pi: int) -> int:
        return self.mi.GetPieceLength(pi)

    def getFileOffset(self, pi: int) -> int:
        return self.mi.PieceLength() * pi

    def Complete(self) -> bool:
        return bool(self.complete.all())

    def _check(self, data, pi: int):
        if pi < 0 or pi >= self.NumPieces():
            raise IndexError(f"invalid piece index {pi}: num pieces = {self.NumPieces()}")
        if len(data) != self.PieceLength(pi):
            raise ValueError(f"invalid piece length: expected {self.PieceLength(pi)}, got {len(data)}")
        if self.complete[pi]:
            raise ErrPieceComplete()

    def _commit(self, data, pi: int):
        with open(self.path, "r+b") as f:
            f.seek(self.getFileOffset(pi))
            f.write(memoryview(data))
        self.complete[pi] = True

    def WritePiece(self, data, pi: int) -> None:
        """torrent.go:203-220 + writePiece :174-199 for one piece."""
        err = self.WritePieces({pi: data})[pi]
        if err is not None:
            raise err

    def WritePieces(self, pieces: dict) -> dict:
        """Verify and write many pieces at once; {pi: None | exception}."""
        out, todo = {}, []
        for pi, data in pieces.items():
            try:
                self._check(data, pi)
                todo.append(pi)
            except (IndexError, ValueError, ErrPieceComplete) as e:
                out[pi] = e
        ok = verify_pieces([pieces[pi] for pi in todo], [self.mi.GetPieceSum(pi) for pi in todo])
        for pi, good in zip(todo, ok):
            if good:
                self._commit(pieces[pi], pi)
                out[pi] = None
            else:
                out[pi] = ValueError("invalid piece sum")
        return out
