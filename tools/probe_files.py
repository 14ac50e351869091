"""Regen from cache files (development probe, not the bench contract): GB/s of
Generator.GenerateBatch over a DirCAS of synthetic files, file route
(krk_piece_sums_files: pread threads / O_DIRECT into pinned windows) vs the reader
route (Python reads into pageable memory, then krk_piece_sums_host).  Warm page
cache: the files were just written."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kraken_amd import core, metainfogen  # noqa: E402
from kraken_amd import device as D  # noqa: E402


class ReaderOnly:
    def __init__(self, cas):
        self.cas = cas

    def GetCacheFileStat(self, h):
        return self.cas.GetCacheFileStat(h)

    def GetCacheFileReader(self, h):
        return self.cas.GetCacheFileReader(h)

    def SetCacheFileMetadata(self, h, mi):
        return self.cas.SetCacheFileMetadata(h, mi)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    D.set_device(0)
    root = tempfile.mkdtemp(dir=a.dir)
    try:
        cas = metainfogen.DirCAS(root)
        base = np.random.default_rng(1).integers(0, 256, size=a.mb << 20, dtype=np.uint8)
        ds = []
        for i in range(a.files):
            base[:8] = np.frombuffer(np.uint64(i).tobytes(), np.uint8)
            d = core.NewSHA256DigestFromHex(f"{i:064x}")
            cas.WriteCacheFileAs(d, base)
            ds.append(d)
        total = a.files * (a.mb << 20)
        cfg = {0: 4 << 20}
        res = {"files": a.files, "mb": a.mb, "fs_dir": root}
        ref = None
        for name, env, c in [("files_pread", "0", cas), ("files_direct", "1", cas), ("reader", "0", ReaderOnly(cas))]:
            os.environ["KRK_FILE_DIRECT"] = env
            g = metainfogen.New(cfg, c)
            mis = g.GenerateBatch(ds)  # warm
            ih = [mi.InfoHash() for mi in mis]
            assert ref is None or ih == ref, name
            ref = ih
            t0 = time.perf_counter()
            for _ in range(a.reps):
                g.GenerateBatch(ds)
            res[name + "_GBps"] = round(total * a.reps / (time.perf_counter() - t0) / 1e9, 2)
        res["outputs_equal"] = True
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
