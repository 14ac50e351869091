"""Host-side mirror of lib/metainfogen over the C ABI.

* ``newPieceLengthConfig`` / ``pieceLengthConfig.get``: lib/metainfogen/config.go:48-80
* ``Generator.Generate``: lib/metainfogen/generator.go:40-58 (stat -> piece length
  -> NewMetaInfo over the cache file -> persist the _torrentmeta sidecar)
* ``Generator.GenerateBatch``: the batch form used for whole-CAS regeneration
  (SURVEY.md §8(f) row 2): one pass over many cache files (krk_piece_sums_files).
* ``Generator.VerifyAndGenerateBatch`` / ``VerifyAndGenerateUploads``: upload verification
  fused with Generate, over upload bytes or the upload files.

The CAS store itself (lib/store) is out of scope; ``DirCAS`` is a minimal
stand-in exposing the three calls Generate makes.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import core
from ._capi import KRK_EIO, check, krk_blob, krk_file_blob, lib


class pieceLengthConfig:
    def __init__(self, ranges):
        self.ranges = ranges  # sorted [(fileSize, pieceLength)]

    def get(self, file_size: int) -> int:
        t = np.ascontiguousarray([a for a, _ in self.ranges], dtype=np.int64)
        l = np.ascontiguousarray([b for _, b in self.ranges], dtype=np.int64)
        return lib.krk_piece_length_for_size(t.ctypes.data_as(C.POINTER(C.c_int64)),
                                              l.ctypes.data_as(C.POINTER(C.c_int64)), len(t), file_size)


def newPieceLengthConfig(piece_length_by_file_size: dict) -> pieceLengthConfig:
    if not piece_length_by_file_size:
        raise ValueError("no piece lengths configured")
    return pieceLengthConfig(sorted((int(a), int(b)) for a, b in piece_length_by_file_size.items()))


DefaultShardIDLength = 2  # lib/store/base/const.go:16-18


class DirCAS:
    """Minimal content-addressed cache directory in the reference's layout:
    <root>/<hex[0:2]>/<hex[2:4]>/<hex>/data with the _torrentmeta sidecar beside it
    (casFileEntryFactory.GetRelativePath, lib/store/base/file_entry.go:176-189;
    getMetadataPath :468-469)."""

    def __init__(self, root: str):
        self.root = root

    def _dir(self, hex_: str) -> str:
        shards = [hex_[2 * i:2 * i + 2] for i in range(min(DefaultShardIDLength, len(hex_) // 2))]
        return os.path.join(self.root, *shards, hex_)

    def ListNames(self) -> list[str]:
        """Every cached blob name, walking the shard directories (file_entry.go ListNames)."""
        out = []
        for dirpath, dirnames, filenames in os.walk(self.root):
            rel = os.path.relpath(dirpath, self.root)
            depth = 0 if rel == "." else rel.count(os.sep) + 1
            if depth == DefaultShardIDLength + 1 and "data" in filenames:
                out.append(os.path.basename(dirpath))
                dirnames[:] = []
        return sorted(out)

    def GetCacheFileStat(self, hex_: str) -> os.stat_result:
        return os.stat(os.path.join(self._dir(hex_), "data"))

    def GetCacheFileReader(self, hex_: str):
        return open(os.path.join(self._dir(hex_), "data"), "rb")

    def GetCacheFilePath(self, hex_: str) -> str:
        """The cache file's path (base FileOp.GetFilePath): lets GenerateBatch read
        the file natively into pinned staging instead of through a reader."""
        return os.path.join(self._dir(hex_), "data")

    def SetCacheFileMetadata(self, hex_: str, mi: core.MetaInfo) -> bool:
        p = os.path.join(self._dir(hex_), "_torrentmeta")
        b = mi.Serialize()
        if os.path.exists(p) and open(p, "rb").read() == b:
            return False
        with open(p, "wb") as f:
            f.write(b)
        return True

    def WriteCacheFileAs(self, d: core.Digest, data) -> core.Digest:
        """Commit already-verified bytes under their digest."""
        os.makedirs(self._dir(d.Hex()), exist_ok=True)
        with open(os.path.join(self._dir(d.Hex()), "data"), "wb") as f:
            f.write(memoryview(data))
        return d

    def MoveUploadFileToCache(self, upload_path: str, hex_: str) -> None:
        """CAStore.MoveUploadFileToCache (origin/blobserver/uploader.go:98 commit): the
        verified upload file renamed into the cache; FileExistsError when the blob is
        already cached (the uploader's 409).  The upload file is deleted either way
        (lib/store/ca_store.go:79-86: `defer s.DeleteUploadFile(uploadName)`)."""
        dst = os.path.join(self._dir(hex_), "data")
        os.makedirs(self._dir(hex_), exist_ok=True)
        try:
            if os.path.exists(dst):
                raise FileExistsError(dst)
            os.replace(upload_path, dst)
        finally:
            if os.path.exists(upload_path):
                os.remove(upload_path)

    def WriteCacheFile(self, data: bytes) -> core.Digest:
        d = core.NewDigester().FromBytes(data)
        os.makedirs(self._dir(d.Hex()), exist_ok=True)
        with open(os.path.join(self._dir(d.Hex()), "data"), "wb") as f:
            f.write(data)
        return d


class Generator:
    def __init__(self, config: dict, cas):
        try:
            self.pieceLengthConfig = newPieceLengthConfig(config)
        except ValueError as e:
            raise ValueError(f"piece length config: {e}") from None
        self.cas = cas

    def Generate(self, d: core.Digest) -> None:
        try:
            info = self.cas.GetCacheFileStat(d.Hex())
        except OSError as e:
            raise IOError(f"cache stat: {e}") from None
        try:
            f = self.cas.GetCacheFileReader(d.Hex())
        except OSError as e:
            raise IOError(f"get cache file: {e}") from None
        with f:
            pl = self.pieceLengthConfig.get(info.st_size)
            try:
                mi = core.NewMetaInfo(d, f, pl)
            except (ValueError, IOError) as e:
                raise IOError(f"create metainfo: {e}") from None
        try:
            self.cas.SetCacheFileMetadata(d.Hex(), mi)
        except OSError as e:
            raise IOError(f"set metainfo: {e}") from None

    def RegenerateAll(self, batch_bytes: int = 8 << 30) -> dict:
        """Whole-CAS regeneration: every cached blob's
        _torrentmeta rewritten from GPU piece sums in batches of ~batch_bytes
        (each batch one pinned, pipelined pass), byte-identical to what
        Generate writes.  Returns counts of blobs seen / sidecars changed."""
        names = self.cas.ListNames()
        seen = changed = 0
        batch, size = [], 0
        for i, name in enumerate(names):
            batch.append(core.NewSHA256DigestFromHex(name))
            size += self.cas.GetCacheFileStat(name).st_size
            if size >= batch_bytes or i == len(names) - 1:
                self.GenerateBatch(batch)
                changed += self._last_changed
                seen += len(batch)
                batch, size = [], 0
        return {"blobs": seen, "changed": changed}

    def GenerateBatch(self, digests) -> list[core.MetaInfo]:
        """Generate for many cache files in one pipelined GPU pass.  When the CAS
        exposes file paths (DirCAS.GetCacheFilePath) the files are read by the
        library's host threads straight into pinned staging windows
        (krk_piece_sums_files); otherwise through GetCacheFileReader into host
        memory (krk_piece_sums_host).  Errors carry Generate's prefixes
        (generator.go:41-58)."""
        if hasattr(self.cas, "GetCacheFilePath"):
            metas, off = [], 0
            for d in digests:
                try:
                    size = self.cas.GetCacheFileStat(d.Hex()).st_size
                except OSError as e:
                    raise IOError(f"cache stat: {e}") from None
                pl = self.pieceLengthConfig.get(size)
                metas.append((d, size, pl, off))
                off += int(lib.krk_num_pieces(size, pl))
            paths = [os.fsencode(self.cas.GetCacheFilePath(d.Hex())) for d, *_ in metas]
            arr = (krk_file_blob * max(len(metas), 1))()
            for i, ((d, size, pl, o), path) in enumerate(zip(metas, paths)):
                arr[i] = krk_file_blob(path, size, pl, o)
            sums = np.zeros(max(off, 1), dtype=np.uint32)
            rc = lib.krk_piece_sums_files(arr, len(metas), sums.ctypes.data_as(C.POINTER(C.c_uint32)))
            if rc == KRK_EIO:
                raise IOError(f"create metainfo: {lib.krk_last_error().decode()}")
            check(rc)
        else:
            datas, metas, off = [], [], 0
            for d in digests:
                try:
                    f = self.cas.GetCacheFileReader(d.Hex())
                except OSError as e:
                    raise IOError(f"get cache file: {e}") from None
                with f:
                    b = np.frombuffer(f.read(), dtype=np.uint8)
                pl = self.pieceLengthConfig.get(b.size)
                datas.append(b)
                metas.append((d, b.size, pl, off))
                off += int(lib.krk_num_pieces(b.size, pl))
            arr = (krk_blob * max(len(metas), 1))()
            for i, (b, (d, size, pl, o)) in enumerate(zip(datas, metas)):
                arr[i] = krk_blob(b.ctypes.data if b.size else None, size, pl, o)
            sums = np.zeros(max(off, 1), dtype=np.uint32)
            check(lib.krk_piece_sums_host(arr, len(metas), sums.ctypes.data_as(C.POINTER(C.c_uint32))))
        out = []
        self._last_changed = 0
        counts = [int(lib.krk_num_pieces(size, pl)) for _, size, pl, _ in metas]
        ihs = core._info_hash_batch([pl for _, _, pl, _ in metas], sums, [o for *_, o in metas], counts,
                                    [d.Hex() for d, *_ in metas], [size for _, size, _, _ in metas])
        for (d, size, pl, o), n, ih in zip(metas, counts, ihs):
            s_ = sums[o:o + n].copy() if n else None
            mi = core.MetaInfo(pl, s_, d.Hex(), size, d, ih)
            try:
                self._last_changed += bool(self.cas.SetCacheFileMetadata(d.Hex(), mi))
            except OSError as e:
                raise IOError(f"set metainfo: {e}") from None
            out.append(mi)
        return out

    def VerifyAndGenerateBatch(self, uploads):
        """Fused upload verification + metainfo generation.

        The reference reads every uploaded blob twice: uploader.verify digests it
        (origin/blobserver/uploader.go:74-94, error "computed digest %s doesn't
        match parameter %s") and Generate later re-reads the committed cache file
        for the piece sums (generator.go:41-58).  Here one host->device pass over
        each blob (krk_metainfo_digest_host) yields both.  uploads: [(core.Digest
        expected, bytes-like data)].  Verified blobs are committed to the CAS with
        their _torrentmeta; returns [MetaInfo | ValueError] in input order."""
        from . import device as D
        datas = [np.frombuffer(memoryview(b), dtype=np.uint8) for _, b in uploads]
        pls = [self.pieceLengthConfig.get(int(x.size)) for x in datas]
        sums, dg = D.metainfo_digest_host(datas, pls)
        out = []
        for (want, _), x, pl, s, g in zip(uploads, datas, pls, sums, dg):
            got = core.NewSHA256DigestFromHex(bytes(g).hex())
            if got != want:
                out.append(ValueError(f"computed digest {got.String()} doesn't match parameter {want.String()}"))
                continue
            d = self.cas.WriteCacheFileAs(want, x)
            out.append((d, pl, s.copy() if s.size else None, int(x.size)))
        return self._commit_metainfo(out)

    def VerifyAndGenerateUploads(self, uploads):
        """The same from the upload FILES, as the origin holds them (uploader.verify reads
        the upload file, origin/blobserver/uploader.go:74-94; commit moves it into the
        cache, :96-105; Generate re-reads the cache file, generator.go:41-58): each file is
        read once by krk_metainfo_digest_files and that read yields the digest AND the piece
        sums.  uploads: [(core.Digest expected, upload file path)].  A file that cannot be
        read fails the batch with uploader.verify's prefixes ("get upload file: ...",
        "calculate digest: read blob: <path>: ..."); a digest mismatch is that upload's
        ValueError; verified files are moved into the CAS with their _torrentmeta.  A verified
        upload whose blob is already cached -- or an earlier upload of the same batch put it
        there -- is that upload's FileExistsError (uploader.commit's 409, uploader.go:96-104),
        its upload file deleted as the reference does, and the batch goes on.  Returns
        [MetaInfo | ValueError | FileExistsError] in input order."""
        from . import device as D
        from ._capi import KrakenError
        paths, sizes = [], []
        for _, p in uploads:
            try:
                sizes.append(os.stat(p).st_size)
            except OSError as e:
                raise IOError(f"get upload file: {e}") from None
            paths.append(p)
        pls = [self.pieceLengthConfig.get(n) for n in sizes]
        try:
            sums, dg = D.metainfo_digest_files(paths, sizes, pls)
        except KrakenError as e:
            raise IOError(f"calculate digest: {e}") from None
        out = []
        for (want, p), n, pl, s, g in zip(uploads, sizes, pls, sums, dg):
            got = core.NewSHA256DigestFromHex(bytes(g).hex())
            if got != want:
                out.append(ValueError(f"computed digest {got.String()} doesn't match parameter {want.String()}"))
                continue
            try:
                self.cas.MoveUploadFileToCache(p, want.Hex())
            except FileExistsError as e:
                out.append(e)  # 409 Conflict for this upload only
                continue
            out.append((want, pl, s.copy() if s.size else None, int(n)))
        return self._commit_metainfo(out)

    def _commit_metainfo(self, out):
        """The committed uploads' InfoHashes in one batched call and their sidecars (entries
        that are errors -- digest mismatch, conflict -- pass through)."""
        ok = [k for k, o in enumerate(out) if isinstance(o, tuple)]
        if ok:
            flat = [out[k][2] for k in ok if out[k][2] is not None]
            allsums = np.concatenate(flat) if flat else np.zeros(0, np.uint32)
            counts = [0 if out[k][2] is None else out[k][2].size for k in ok]
            offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint64)
            ihs = core._info_hash_batch([out[k][1] for k in ok], allsums, offs, counts,
                                        [out[k][0].Hex() for k in ok], [out[k][3] for k in ok])
            for k, ih in zip(ok, ihs):
                d, pl, s, size = out[k]
                mi = core.MetaInfo(pl, s, d.Hex(), size, d, ih)
                self.cas.SetCacheFileMetadata(d.Hex(), mi)
                out[k] = mi
        return out


def New(config: dict, cas) -> Generator:
    return Generator(config, cas)


def _parse_config(text: str) -> dict:
    """"0:4194304,2147483648:8388608" -> {0: 4194304, 2147483648: 8388608}."""
    out = {}
    for part in text.split(","):
        a, b = part.split(":")
        out[int(a)] = int(b)
    return out


def main(argv=None) -> int:
    """python -m kraken_amd.metainfogen <cache dir> [--piece-lengths 0:4194304]:
    regenerate every _torrentmeta of a CAS cache directory on the GPU."""
    import argparse
    import json
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("cache_dir")
    ap.add_argument("--piece-lengths", default="0:4194304",
                    help="size:pieceLength ranges (config/origin/base.yaml:24-26 default: 0:4MB)")
    ap.add_argument("--batch-gib", type=int, default=8)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    from . import device
    device.set_device(a.device)
    g = New(_parse_config(a.piece_lengths), DirCAS(a.cache_dir))
    print(json.dumps(g.RegenerateAll(a.batch_gib << 30)))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
