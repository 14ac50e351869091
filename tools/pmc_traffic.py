"""Per-launch HBM traffic from rocprofv3 PMC counter CSVs -> profiles/pmc_traffic.json.

Collect FETCH_SIZE and WRITE_SIZE in SEPARATE passes (they do not fit one pass on
gfx950), each with only --kernel-trace/--stats beside --pmc, e.g.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- python bench.py ...

Corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming
read (128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  Both are per dispatch and summed over the 8 XCDs by the tool.
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict

KERNELS = {"crc_items_kernel": "crc32_pieces", "gather_kernel": "host_gather", "sha256_ws_kernel": "sha256_multi", "sha256_w8_kernel": "sha256_multi",
           "sha256_multi_kernel": "sha256_multi", "hrw_order_kernel": "hrw_order",
           "shard_gather_kernel": "hrw_gather", "shard_gather_packed_kernel": "hrw_gather",
           "pack_owner_rows_kernel": "hrw_order", "synth_fill": "synth_fill"}


def _short(name: str):
    for k, v in sorted(KERNELS.items(), key=lambda kv: -len(kv[0])):  # the longest name first
        if k in name:
            return v
    return None


def read_counter(dirpath: str, counter: str):
    """{kernel: [value per dispatch]} for one counter from a rocprofv3 output dir."""
    out = defaultdict(list)
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        per_dispatch = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per_dispatch[d] += float(row["Counter_Value"])
                names[d] = row.get("Kernel_Name", "")
        for d, v in per_dispatch.items():
            k = _short(names[d])
            if k:
                out[k].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True, help="rocprofv3 output dir of the FETCH_SIZE pass")
    ap.add_argument("--write", required=True, help="rocprofv3 output dir of the WRITE_SIZE pass")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--blobs", type=int, default=1000)
    ap.add_argument("--algorithmic-bytes", type=float, default=1000 * 104857600.0)
    ap.add_argument("--pick", default="median", choices=["median", "max"],
                    help="a kernel's dispatches: the median, or the largest (the workload's own launch "
                         "when the run has shorter ones of the same kernel)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    res = {"workload": a.workload, "blobs": a.blobs, "algorithmic_bytes_per_launch": a.algorithmic_bytes,
           "dispatch": a.pick,
           "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "bytes_per_launch": {}, "raw": {}}
    for k in sorted(set(fetch) | set(write)):
        agg = max if a.pick == "max" else statistics.median
        f = agg(fetch[k]) if fetch.get(k) else 0.0
        w = agg(write[k]) if write.get(k) else 0.0
        b = 2 * f * 1024 + w * 1024
        res["bytes_per_launch"][k] = b
        res["raw"][k] = {"FETCH_SIZE_KiB_median": f, "WRITE_SIZE_KiB_median": w,
                         "dispatches": [len(fetch.get(k, [])), len(write.get(k, []))],
                         "traffic_over_algorithmic": b / a.algorithmic_bytes if a.algorithmic_bytes else None}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
