"""Debug probe: device SHA-256 of a few short blobs through the current library
(KRK_LIB_PATH selects an experiment build); prints H0..H7 of each digest."""
import hashlib
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from kraken_amd import device as D  # noqa: E402
from oracle import oracle as orc  # noqa: E402

D.set_device(0)
lens = [0, 1, 56, 64, 130, 1000]
arena = D.BlobArena(lens, 4096, blob_ids=range(len(lens)))
out = D.BatchOutputs(arena)
D.sha256(arena, out)
D.synchronize()
got = out.digests.to_host(np.uint8, 32 * len(lens)).reshape(-1, 32)
for i, L in enumerate(lens):
    ref = hashlib.sha256(orc.synth(i, L).tobytes()).digest()
    print(L, bytes(got[i]).hex()[:32], ref.hex()[:32], "ok" if bytes(got[i]) == ref else "BAD")
