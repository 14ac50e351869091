"""Every C3 blob against the oracle: the bench's C3 workload (20,000 blobs of the BASELINE law,
11.75 TB, 4 MiB pieces) through the production windowed GPU path once (kraken_amd.windowed
WindowedRun, GPU only, the bench's 48 GiB windows), then each blob regenerated on the host and
hashed by the CPU oracle (oracle/oracle.c: SHA-256 pass + CRC-32 piece pass, one blob per
thread), and every digest and every piece sum compared.

The -m gpu tests check C3 at full lengths on a 256-blob sample and rank 0's whole 8-GPU shard;
this one-off run covers the whole config (the oracle needs ~10 minutes of a 16-core host, too
long for the test suite).  Writes gpurun_out/c3_full_oracle.json; prints a progress line per
oracle chunk.

    python tools/c3_full_oracle.py [--threads 16] [--chunk 1000] [--blobs 20000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=1000, help="blobs per oracle call")
    ap.add_argument("--blobs", type=int, default=None, help="C3 law over this many blobs (default 20,000)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c3_full_oracle.json"))
    a = ap.parse_args()

    import bench
    from kraken_amd import device as D
    from kraken_amd.windowed import WindowedRun
    from oracle import oracle as O

    ids, lens, P = bench.workload_blobs("c3", 0, 1, a.blobs)
    n = len(lens)
    D.set_device(0)
    D.set_sha_host_offload(0)  # every chain on the GPU
    t0 = time.perf_counter()
    wr = WindowedRun(D, ids, lens, P, 48 << 30)
    try:
        wr.run()
        gpu_s = time.perf_counter() - t0
        cb = wr.cb
        dg = cb.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
        sums = cb.sums.to_host(np.uint32, cb.total_pieces)
        offs = np.asarray(cb.sums_off, dtype=np.int64).copy()
        windows = len(wr.wins)
    finally:
        wr.close()
    total = int(sum(lens))
    print(f"gpu: {n} blobs, {total / 1e12:.3f} TB, {windows} windows, {gpu_s:.1f} s", flush=True)

    bad_dg, bad_sums, pieces = [], [], 0
    t1 = time.perf_counter()
    for c0 in range(0, n, a.chunk):
        c1 = min(n, c0 + a.chunk)
        _, dgo, (so, offo) = O.baseline_run_lazy(ids[c0:c1], lens[c0:c1], P, a.threads, passes=3)
        for k in range(c1 - c0):
            b = c0 + k
            if not np.array_equal(dgo[k], dg[b]):
                bad_dg.append(b)
            m = int(offo[k + 1] - offo[k])
            pieces += m
            if not np.array_equal(sums[offs[b]:offs[b] + m], so[int(offo[k]):int(offo[k + 1])]):
                bad_sums.append(b)
        done = int(sum(lens[:c1]))
        el = time.perf_counter() - t1
        print(f"oracle: {c1}/{n} blobs, {done / 1e12:.3f} TB, {el:.0f} s, mismatches digest {len(bad_dg)} "
              f"sums {len(bad_sums)}", flush=True)
    res = {"what": "every C3 blob's digest and piece sums from the GPU windowed path (GPU only) against the CPU "
                   "oracle (oracle/oracle.c) over the same seeded bytes regenerated on the host",
           "blobs": n, "bytes": total, "pieces": pieces, "piece_length": P, "windows": windows,
           "gpu_run_s": round(gpu_s, 2), "oracle_s": round(time.perf_counter() - t1, 1), "oracle_threads": a.threads,
           "digest_mismatches": bad_dg[:50], "n_digest_mismatches": len(bad_dg),
           "sum_mismatches": bad_sums[:50], "n_sum_mismatches": len(bad_sums),
           "all_equal": not bad_dg and not bad_sums, "longest_blob": int(max(lens)), "shortest_blob": int(min(lens))}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res), flush=True)
    sys.exit(0 if res["all_equal"] else 1)


if __name__ == "__main__":
    main()
