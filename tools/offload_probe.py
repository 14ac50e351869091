"""SHA-256 host offload (krk_set_sha_host_offload) on the c5regen_digest batch at several
host thread counts: wall time of krk_metainfo_digest_dev and the planner's split
(development tool; KRK_TRACE=1 adds the per-call wait / hash split on stderr)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kraken_amd import device as D  # noqa: E402


def main():
    D.set_device(0)
    ids, lens, P = bench.workload_blobs(os.environ.get("WORKLOAD", "c5regen_digest"), 0, 1, 0)
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    for T in [int(x) for x in os.environ.get("THREADS", "16,14,12,8").split(",")]:
        idx, g, h = D.sha_offload_plan(lens, T)
        D.set_sha_host_offload(T)
        walls = []
        for _ in range(2):
            t0 = time.perf_counter()
            D.metainfo_digest(arena, out)
            D.synchronize()
            walls.append(time.perf_counter() - t0)
        D.set_sha_host_offload(0)
        print(json.dumps({"threads": T, "blobs_on_host": int(idx.size), "model_gpu_s": round(g, 3),
                          "model_host_s": round(h, 3), "wall_s": [round(w, 3) for w in walls],
                          "GBps": round(sum(lens) / min(walls) / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
