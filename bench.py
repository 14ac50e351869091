#!/usr/bin/env python
"""bench.py -- metainfo+digest GB/s on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "C2"): 1,000 synthetic 100 MiB
blobs, 4 MiB pieces, resident in HBM.  One step = the hot path over the batch:
the piece CRC-32 of every piece (core.calcPieceSums) and the whole-blob SHA-256
of every blob (core.Digester), both through the C ABI (krk_metainfo_digest_dev:
the SHA and CRC kernels run concurrently on two streams), with the 25,000 sums
and the 1,000 digests copied back to the host inside the step.

Other configs of BASELINE.json (--workload): c1 (one 1 GiB blob), c3 (this
rank's LPT shard of 20k blobs of 100 MiB-1 GiB, streamed through HBM in
windows with krk_metainfo_digest_chunks_dev; the synthetic window generation
runs on its own stream, overlapped, inside the timed region), c4 (one 20 GiB
blob, 256 KiB pieces, piece sums only), c5 (1M-digest hashring placement,
digests/s) and c5regen (1,000 blobs of log-uniform sizes with the metainfogen
piece-length ranges).

Multi-GPU: one process per GPU (torch.distributed.run); the path shards by blob
with no data-path collective (C2 is weak scaling: every rank runs its own 1,000
blobs, ids offset by rank; C3 is a fixed total split by LPT).  A gloo barrier
brackets the timed region, the time is the max over ranks, and value = units
processed by all ranks / that time.

cpu_baseline (rank 0, N=1): the CPU restatement of the reference's path
(oracle/: the two-pass SHA-NI + PCLMUL run, or the HRW ring placement) on the
host cores of this box, on a bounded sample of the same synthetic inputs.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kraken_amd.windowed import c3_lengths  # noqa: E402

METRIC = "metainfo+digest GB/s (device-resident & end-to-end) at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1

# Per-stream SHA-256 issue ceiling, from the ISA and the clock:
# the VALU instructions per block of the production consumer loop, counted in the
# disassembly of the loaded library's gfx950 code object (tools/sha_isa.py), each
# costing >= 4 cycles for a wave alone on its SIMD (MI355X_MICROARCH.md 'vector-
# instruction ISSUE cost'), at the shader clock measured by a probe kernel that
# runs beside a SHA-256 launch (krk_device_clock_mhz).
sys.path.insert(0, os.path.join(ROOT, "tools"))


def sha_isa_ceiling(D, launch, lanes):
    """(isa counts, clock MHz, per-stream ceiling MB/s); launch() starts one SHA-256
    batch asynchronously, the clock is read while it runs."""
    import ctypes as C
    import sha_isa
    try:
        isa = sha_isa.count(D.lib._name, lanes)
    except Exception as e:  # tools missing on the box: report, never guess
        return {"error": f"{type(e).__name__}: {e}"}, None, None
    s = C.c_void_p()
    D.check(D.lib.krk_stream_create(C.byref(s)))
    mhz = C.c_double()
    launch()
    time.sleep(0.3)  # inside the launch (C2: ~2 s)
    D.check(D.lib.krk_device_clock_mhz(s, C.byref(mhz)))
    D.synchronize()
    D.lib.krk_stream_destroy(s)
    return isa, mhz.value, sha_isa.ceiling_mbps(isa, mhz.value)


def load_valu(workload):
    """VALU / LDS utilisation per kernel from the committed rocprofv3 PMC passes
    (tools/pmc_valu.py -> profiles/r03/valu_<workload>.json); the raw counters stay in
    that file, the derived fractions go into the bench line."""
    d, path = None, None
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # the newest round's passes
        path = os.path.join(ROOT, "profiles", rnd, f"valu_{workload}.json")
        try:
            d = json.load(open(path))
            break
        except (OSError, ValueError):
            d = None
    if d is None:
        return {}, None
    keep = ("valu_issue_frac_per_wave", "valu_busy_chip_pct", "lds_issue_frac_per_wave", "lds_bank_conflict_frac",
            "wait_any_frac_per_wave", "wait_inst_any_frac_per_wave", "clock_mhz", "kernel_ms", "dispatches")
    out = {}
    for mode in ("device_resident", "end_to_end"):
        out[mode] = {k: {m: v[m] for m in keep if m in v} for k, v in d.get(mode, {}).items() if isinstance(v, dict)}
    return out, os.path.relpath(path, ROOT)


WORKLOADS = {
    "c2": dict(kind="metainfo", desc="C2: 1000 x 100 MiB blobs, 4 MiB pieces, piece CRC-32 + SHA-256 per blob"),
    "c1": dict(kind="metainfo", desc="C1: 1 x 1 GiB blob, 4 MiB pieces (one SHA-256 stream)"),
    "small": dict(kind="metainfo", desc="dev: 64 x 16 MiB blobs, 4 MiB pieces"),
    "c5regen": dict(kind="regen", desc="C5 regen: Generator.Generate over 1000 blobs (piece sums + InfoHash, no "
                                       "digest: core/metainfo.go:53-55), log-uniform sizes in [0, 1 GiB), piece "
                                       "lengths from {0:1MB, 2GB:4MB, 4GB:8MB}"),
    "c5regen_digest": dict(kind="metainfo", desc="C5 regen blobs with the upload digest as well (metainfo + "
                                                 "SHA-256 per blob)"),
    # warmup 3: the host/GPU split's learning calls (window setup, a split sample, a host-only
    # sample) run before the timed steps, as in a long-running agent
    "f1verify": dict(kind="verify", steps=5, warmup=3, desc="Agent piece verify (agentstorage.Torrent.writePiece, torrent.go:174-199): "
                                         "4,096 received 4 MiB pieces in pinned host receive buffers checked against "
                                         "GetPieceSum, split between host threads and the GPU; 1 in 64 corrupted"),
    "c4": dict(kind="pieces", steps=20, warmup=2,  # 3.6 ms steps
               desc="C4: one 20 GiB blob per GPU, 256 KiB pieces (81,920), piece sums only"),
    "c3": dict(kind="chunked", desc="C3: 20k blobs of 100 MiB + (rng mod 968,884,225) B, 4 MiB pieces, "
                                    "LPT-sharded by blob, streamed through HBM in windows"),
    "engine": dict(kind="engine", steps=3, warmup=1,
                   desc="256 concurrent GPU Digesters (core.Digester per upload / cache fill, "
                        "origin/blobserver/uploader.go:75) on 256 native threads, 16 MiB each in random writes of "
                        "up to 1 MiB (tests/native/digesters.cpp, a C-ABI caller like the cgo layer)"),
    "files": dict(kind="files", steps=3, warmup=1,
                  desc="upload / cache-fill verify + metainfo from CAS files (uploader.go:74-94 + generator.go:41-58):"
                       " 16,384 blobs of the C3 length law / 64 (1.6-16.8 MB, 151 GB a pass), each a prefix of one of"
                       " 64 source files, 4 MiB pieces; every byte read once (pread -> pinned windows -> PCIe)"),
    "defaults": dict(kind="defaults", steps=3, warmup=0,
                     desc="the library's defaults, no knobs: one 1 GiB blob (C1) through krk_metainfo_digest_dev "
                          "and one 1 GiB NewMetaInfo piece stream of 4 MiB reads, each against one host thread"),
    "c5": dict(kind="hrw", steps=50, warmup=5,  # 0.4 ms steps: a few would time launch jitter
               desc="C5: 1M seeded 32-B digests -> hashring.Locations (ShardID key), "
                    "16 origins weight 100, MaxReplica 3, all healthy"),
}


def _env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def host_budget():
    """(this rank's host CPU budget, the node's CPUs, where the budget came from), from the
    library itself (krk_host_cpu_budget: KRK_HOST_CPUS, else the node's CPUs -- affinity
    capped by the cgroup quota -- divided among LOCAL_WORLD_SIZE ranks, else capped by
    OMP_NUM_THREADS), so the bench's host legs size themselves as the library does."""
    from kraken_amd import _capi
    return _capi.host_cpu_budget()


def host_cores() -> int:
    """CPUs this rank's host legs may use: the library's per-process budget."""
    return host_budget()[0]


def node_cores() -> int:
    """All of the node's host cores (GOMAXPROCS = every core, BASELINE.json north_star):
    what rank 0's cpu_baseline runs on at every N, whatever a launcher put in
    OMP_NUM_THREADS.  The other ranks wait at a barrier meanwhile."""
    return host_budget()[1]


def baseline_sample_blobs() -> int:
    """Blobs in a CPU baseline sample: one per core at least (one goroutine a blob, every
    core busy), two per core up to 32 (load balance on small nodes)."""
    return max(node_cores(), min(2 * node_cores(), 32))


CORES_SOURCE = ("the node's host cores: affinity capped by the cgroup cpu.max quota (krk_host_cpu_budget "
                "node_cpus; OMP_NUM_THREADS and LOCAL_WORLD_SIZE not applied)")


# ----------------------------------------------------------------- workloads
def c5regen_lengths(n=1000):
    """Log-uniform in [0, 2^30): L = floor(2^(30*u)) - 1, u from a seeded stream."""
    out = []
    for i in range(n):
        u = (mix64((0xC5 + i * GAMMA) & M64) >> 11) / float(1 << 53)
        out.append(int(math.floor(2.0 ** (30.0 * u))) - 1)
    return out


def workload_blobs(name, rank, world, nblobs_override):
    """(blob ids, lengths, piece length) this rank processes."""
    if name == "c2":
        n = nblobs_override or 1000
        return [rank * n + i for i in range(n)], [100 << 20] * n, 4 << 20
    if name == "c1":
        return [rank], [1 << 30], 4 << 20
    if name == "small":
        n = nblobs_override or 64
        return [rank * n + i for i in range(n)], [16 << 20] * n, 4 << 20
    if name == "c4":
        return [rank], [20 << 30], 256 << 10
    if name in ("c5regen", "c5regen_digest"):
        from kraken_amd import metainfogen
        lens = c5regen_lengths(nblobs_override or 1000)
        cfg = metainfogen.newPieceLengthConfig({0: 1 << 20, 2 << 30: 4 << 20, 4 << 30: 8 << 20})
        pls = {cfg.get(L) for L in lens}
        assert len(pls) == 1, pls  # every C5 regen blob is < 2 GB -> 1 MiB pieces
        ids = [(1 << 40) + rank * len(lens) + i for i in range(len(lens))]
        return ids, lens, pls.pop()
    if name == "c3":
        from kraken_amd.shard import lpt_shard
        lens = c3_lengths(nblobs_override or 20000)
        mine = lpt_shard(lens, world)[rank]
        return [(2 << 40) + i for i in mine], [lens[i] for i in mine], 4 << 20
    raise ValueError(name)


# -------------------------------------------------------------- CPU baseline
def cpu_baseline_metainfo(lens_sample, ids_sample, piece, target_s, passes=3):
    from oracle import oracle as O  # the CPU baseline leg (test infrastructure)
    O.build()
    # one blob per worker, as the reference (one goroutine per blob): C1's single blob is one core
    threads = min(node_cores(), len(lens_sample))
    t1, dg, sums = O.baseline_run(ids_sample, lens_sample, piece, threads, fast=True, want_outputs=True,
                                  passes=passes)
    reps = max(1, int(round(target_s / max(t1, 1e-3))))
    t, _, _ = O.baseline_run(ids_sample, lens_sample, piece, threads, fast=True, repeats=reps, passes=passes)
    total = sum(lens_sample) * reps
    what = {3: "SHA-256 pass (SHA-NI) then CRC-32 piece pass (PCLMUL)", 2: "CRC-32 piece pass (PCLMUL) only",
            1: "SHA-256 pass (SHA-NI) only"}[passes]
    src = CORES_SOURCE if threads == node_cores() else (
        f"one thread per blob, as the reference's one goroutine per blob: min({node_cores()} node cores "
        f"({CORES_SOURCE}), {len(lens_sample)} blobs)")
    info = {"value": round(total / t / 1e9, 3), "unit": "GB/s", "cores": threads, "cores_source": src,
            "kind": "port",
            "sample": (f"{len(lens_sample)} synthetic blobs ({sum(lens_sample) / 2**20:.0f} MiB) x {reps} passes "
                       f"({t:.1f} s): {what}, 32 KiB chunks, one blob per thread, {threads} threads "
                       f"({'the host node' if threads == node_cores() else 'of the host node'}'s cores), "
                       "oracle/oracle.c"),
            "seconds": round(t, 2), "have_shani": bool(O.lib().orc_have_shani()),
            "have_clmul": bool(O.lib().orc_have_clmul())}
    return info, dg, sums


C3_CPU_SAMPLE = 256


def cpu_baseline_c3(ids, lens, P, dg_gpu, sums_gpu, sums_off_gpu):
    """C3's CPU baseline (a seeded 256-blob subset, GB/s): the reference's
    two passes per blob (origin/blobserver/uploader.go:74-94 digest, then
    lib/metainfogen/generator.go:41-58 piece sums) on every host core, one blob per
    thread.  The sample's blobs (100 MiB - 1 GiB each, ~150 GB) cannot all be held, so
    each thread materialises its next blob untimed in its own buffer and times only the
    passes (oracle orc_baseline_run_lazy); rate = bytes / (summed busy time / threads).
    Every sampled blob's digest and piece sums are compared with the GPU run's."""
    from oracle import oracle as O  # the CPU baseline leg (test infrastructure)
    O.build()
    n = len(lens)
    m = min(n, C3_CPU_SAMPLE)
    pick = np.sort(np.random.default_rng(0xC3).choice(n, m, replace=False))
    threads = min(node_cores(), m)
    lens_s = [int(lens[i]) for i in pick]
    busy, dgc, (s, off) = O.baseline_run_lazy([ids[i] for i in pick], lens_s, P, threads)
    ok = True
    for k, i in enumerate(pick):
        o, cnt = int(sums_off_gpu[i]), int(off[k + 1] - off[k])
        ok = ok and bytes(dgc[k]) == bytes(dg_gpu[i]) and np.array_equal(s[int(off[k]):int(off[k + 1])],
                                                                         sums_gpu[o:o + cnt])
    total = sum(lens_s)
    wall = busy / threads
    return {"value": round(total / wall / 1e9, 3), "unit": "GB/s", "cores": threads, "cores_source": CORES_SOURCE,
            "kind": "port",
            "sample": (f"{m} seeded C3 blobs ({total / 1e9:.1f} GB, {min(lens_s) >> 20}-{max(lens_s) >> 20} MiB): "
                       "SHA-256 pass (SHA-NI) then CRC-32 piece pass (PCLMUL), 32 KiB chunks, one blob per thread, "
                       f"{threads} threads; each blob generated untimed into its thread's buffer, rate = bytes / "
                       f"(summed busy {busy:.1f} s / threads), oracle/oracle.c"),
            "seconds": round(wall, 2), "have_shani": bool(O.lib().orc_have_shani()),
            "have_clmul": bool(O.lib().orc_have_clmul()), "outputs_match_gpu": bool(ok),
            "blobs_checked_against_gpu": int(m)}


def cpu_baseline_hrw(digests, labels, healthy, max_replica, target_s):
    from oracle import oracle as O  # the CPU baseline leg (test infrastructure)
    O.build()
    threads = node_cores()
    m = min(len(digests), 100_000)
    t1, locs, counts = O.baseline_hrw(digests[:m], labels, healthy, max_replica, threads)
    reps = max(1, int(round(target_s / max(t1, 1e-3))))
    t = 0.0
    for _ in range(reps):
        t += O.baseline_hrw(digests[:m], labels, healthy, max_replica, threads)[0]
    return ({"value": round(m * reps / t, 1), "unit": "digests/s", "cores": threads, "cores_source": CORES_SOURCE,
             "kind": "port",
             "sample": f"{m} digests x {reps} passes ({t:.1f} s): GetOrderedNodes(ShardID) + Locations filter "
                       f"per digest, {threads} threads, oracle/oracle.c"}, locs, counts)


# ------------------------------------------------------------------ runners
class Timer:
    def __init__(self, D, dist):
        self.D, self.dist = D, dist
        self.rank_s = None  # every rank's own time of the leg's timed region

    def timed_region(self, x):
        """The leg's timed region: every rank's own seconds (kept for the line's rank_ms),
        the max over ranks returned."""
        if self.dist is None:
            self.rank_s = [x]
            return x
        import torch
        parts = [torch.zeros(1, dtype=torch.float64) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(parts, torch.tensor([x], dtype=torch.float64))
        self.rank_s = [float(p.item()) for p in parts]
        return max(self.rank_s)

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(out, obj)
        return out

    def barrier(self):
        self.D.synchronize()
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


TRAFFIC_SOURCE = ("rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this workload committed under profiles/ "
                  "(tools/pmc_traffic.py): NOT measured in this run (counters need their own profiler process)")
VALU_NOTE = "rocprofv3 PMC passes committed under profiles/ (tools/pmc_valu.py): NOT measured in this run"


def roofline_obj(kernel, gbps, avg_ms, bytes_launch, traffic):
    r = {"kernel": kernel, "bound": "hbm", "achieved": round(gbps, 4), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(gbps / HBM_PEAK_GBPS, 5), "traffic": traffic, "avg_launch_ms": round(avg_ms, 3),
         "algorithmic_bytes_per_launch": bytes_launch}
    if traffic is not None:
        r["traffic_source"] = TRAFFIC_SOURCE
    return r


def sha_roofline(a, D, n, lens, gbps, avg_ms, bytes_launch, traffic, launch):
    """sha256_multi against the HBM roofline the contract prices every kernel on (peak = the
    8 TB/s spec, frac = achieved / peak: ~0.007, VERDICT r05 weak #2 -- the headline shows
    it).  What actually bounds it is per-stream VALU issue (one sequential Merkle-Damgard
    chain per blob): `issue_bound` / `valu` give the streams x ISA per-stream ceiling and the
    fraction of it, beside the HBM one."""
    lanes = D.sha_lanes_per_stream(n)
    per_stream = max(lens) / (avg_ms / 1e3) / 1e6
    roof = {"kernel": "sha256_multi", "bound": "hbm", "achieved": round(gbps, 4),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 5), "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 3), "algorithmic_bytes_per_launch": bytes_launch,
            "valu": {"peak": None, "unit": "GB/s", "frac": None}}
    if traffic is not None:
        roof["traffic_source"] = TRAFFIC_SOURCE
    ib = {"achieved_per_stream_MBps": round(per_stream, 2), "streams": n, "lanes_per_stream": lanes}
    if lanes in (2, 8) and not a.no_ceiling:
        isa, mhz, ceil = sha_isa_ceiling(D, launch, lanes)
        if ceil:
            ib.update({"ceiling_per_stream_MBps": round(ceil, 2), "frac": round(per_stream / ceil, 4),
                       "clock_mhz": round(mhz, 1), "valu_per_block": isa["valu_per_block"],
                       "round_valu_per_block": isa["round_valu_per_block"],
                       "lds_per_block": isa["lds_per_block"], "salu_per_block": isa["salu_per_block"],
                       "ceiling_source": ("ISA: VALU instructions per 64-byte block in the production consumer "
                                          "loop (llvm-objdump of the loaded code object, tools/sha_isa.py) x 4 "
                                          "cycles per VALU for a lone wave (MI355X_MICROARCH.md:489) at the "
                                          "shader clock measured beside a SHA launch (krk_device_clock_mhz)")})
            peak = n * ceil / 1e3
            roof["valu"] = {"peak": round(peak, 4), "unit": "GB/s", "frac": round(gbps / peak, 4),
                            "what": "streams x the ISA per-stream ceiling (issue_bound)"}
            import sha_isa
            fc = sha_isa.fetch_ceiling_mbps(isa, mhz)
            ib["fetch_bound"] = {"code_bytes_per_block": isa["code_bytes_per_block"],
                                 "fetch_bytes_per_cycle": round(sha_isa.FETCH_BYTES_PER_CYCLE, 3),
                                 "ceiling_per_stream_MBps": round(fc, 2), "frac": round(per_stream / fc, 4),
                                 "source": "one wave's code fetch, measured: 8-byte encodings issue every 4.64 "
                                           "cycles whatever the operands (tools/micro/vopcost.hip, "
                                           "profiles/r02/micro_vop_encoding_cost.txt)"}
        else:
            ib["ceiling_error"] = isa.get("error")
    roof["issue_bound"] = ib
    waves = -(-n // (64 // lanes)) if lanes in (2, 8) else -(-n // 64)
    roof["note"] = (f"peak/frac: the HBM roofline (8 TB/s spec). SHA-256 is one sequential Merkle-Damgard chain per "
                    f"blob ({lanes} lane(s) each here), so the kernel is bound by the per-stream VALU issue of its "
                    f"consumer waves ({waves} of the chip's 1,024 SIMDs for {n:,} streams), far below HBM: valu.frac = "
                    "achieved / (streams x ISA per-stream ceiling); fetch_bound = the same loop priced by its code "
                    "bytes (DESIGN.md 4.2)")
    return roof


def load_traffic(path, workload, n):
    """Per-launch HBM bytes from the PMC passes (tools/pmc_traffic.py): `path` if given, else
    the newest of profiles/r06, r05 and r04/pmc_traffic_<workload>.json, profiles/pmc_traffic_<workload>.json
    and (C2) profiles/pmc_traffic.json -- the first whose workload and blob count match."""
    cands = [path] if path else []
    cands += [os.path.join(ROOT, "profiles", "r06", f"pmc_traffic_{workload}.json"),
              os.path.join(ROOT, "profiles", "r05", f"pmc_traffic_{workload}.json"),
              os.path.join(ROOT, "profiles", "r04", f"pmc_traffic_{workload}.json"),
              os.path.join(ROOT, "profiles", f"pmc_traffic_{workload}.json"),
              os.path.join(ROOT, "profiles", "pmc_traffic.json")]
    for c in cands:
        try:
            pm = json.load(open(c))
        except (ValueError, OSError):
            continue
        if pm.get("workload") == workload and pm.get("blobs") == n:
            TRAFFIC_FOUND[workload] = os.path.relpath(c, ROOT)
            return pm.get("bytes_per_launch", {})
    return {}


TRAFFIC_FOUND = {}  # workload -> the committed PMC file load_traffic used


def run_metainfo(a, D, T, rank, world, res):
    ids, lens, P = workload_blobs(a.workload, rank, world, a.blobs)
    n = len(lens)
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    pin_s = D.PinnedArray((max(arena.total_pieces, 1),), np.uint32)  # results gathered to pinned host memory
    pin_d = D.PinnedArray((max(n, 1) * 32,), np.uint8)
    sums_h, dg_h = pin_s.a, pin_d.a

    def step():
        D.metainfo_digest(arena, out)
        D.synchronize()
        pin_s.fill_from(out.sums)
        pin_d.fill_from(out.digests)

    if a.e2e_only:  # profiler passes of the host path: no device-resident launch in the trace
        res.update({"metric": METRIC + " (end-to-end leg only)", "unit": "GB/s", "steps": 1,
                    "end_to_end": end_to_end(D, T, arena, n, min(a.e2e_mb << 20, lens[0]), P, None, world)})
        res["value"] = res["end_to_end"]["value"]
        return
    for _ in range(a.warmup):
        step()
    T.barrier()
    with D.KernelTimer():
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        T.barrier()
        t1 = time.perf_counter()
        crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
        sha_n, sha_ms = D.KernelTimer.stats("sha256_multi")
    elapsed = T.timed_region(t1 - t0)
    bytes_rank = int(sum(lens))
    value = world * bytes_rank * a.steps / elapsed / 1e9
    crc_avg, sha_avg = crc_ms / max(crc_n, 1), sha_ms / max(sha_n, 1)
    crc_gbps = bytes_rank / (crc_avg / 1e3) / 1e9 if crc_n else 0.0
    sha_gbps = bytes_rank / (sha_avg / 1e3) / 1e9 if sha_n else 0.0
    traffic = load_traffic(a.pmc_json, a.workload, n)
    dominant = "sha256_multi" if sha_avg >= crc_avg else "crc32_pieces"
    roof = roofline_obj(dominant, sha_gbps if dominant == "sha256_multi" else crc_gbps,
                        sha_avg if dominant == "sha256_multi" else crc_avg, bytes_rank, traffic.get(dominant))
    roof_crc = roofline_obj("crc32_pieces", crc_gbps, crc_avg, bytes_rank, traffic.get("crc32_pieces"))
    roof_crc["note"] = ("launched together with sha256_multi (krk_metainfo_digest_dev), so it runs on the CUs the "
                        "SHA workgroups leave free (their LDS rings keep a CRC workgroup off a CU that holds one) "
                        "and its time is hidden inside the SHA launch; alone on the chip it is the C4 line "
                        "(DESIGN.md 4.1)")
    valu, valu_src = load_valu(a.workload)
    if valu_src and valu.get("device_resident", {}).get("crc32_pieces"):
        roof_crc["valu"] = dict(valu["device_resident"]["crc32_pieces"], source=valu_src, measured_in_this_run=False,
                               note=VALU_NOTE)
    if dominant == "sha256_multi":
        roof = sha_roofline(a, D, n, lens, sha_gbps, sha_avg, bytes_rank, traffic.get("sha256_multi"),
                            lambda: D.metainfo_digest(arena, out))
    if valu_src and valu.get("device_resident", {}).get(dominant):
        roof["valu"] = dict(valu["device_resident"][dominant], source=valu_src, measured_in_this_run=False,
                            note=VALU_NOTE)
    res.update({"metric": METRIC, "value": round(value, 3), "unit": "GB/s", "steps": a.steps,
                "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "dtype": "u8",
                "data": "synthetic (device-generated splitmix64 blobs, spec in DESIGN.md)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "blobs_per_gpu": n,
                           "bytes_per_gpu": bytes_rank, "piece_length": P, "mode": "device-resident",
                           "parallelism": f"blob-sharded x{world}, no collective"},
                "roofline": roof,
                "roofline_crc": roof_crc,
                "kernels": {"crc32_pieces": {"launches": crc_n, "avg_ms": round(crc_avg, 3)},
                            "sha256_multi": {"launches": sha_n, "avg_ms": round(sha_avg, 3)}}})
    if a.workload in ("c1", "c2", "c5regen_digest") and not a.no_offload:
        res["host_offload"] = host_offload_leg(a, D, T, step, lens, world, dg_h, n)
    if a.workload == "c2" and not a.no_e2e:
        res["end_to_end"] = end_to_end(D, T, arena, n, min(a.e2e_mb << 20, lens[0]), P, out, world)
        ev = valu.get("end_to_end") if valu_src else None
        if ev:
            res["end_to_end"]["valu"] = {"sha256_multi": ev.get("sha256_multi"), "crc32_pieces": ev.get("crc32_pieces"),
                                         "source": valu_src, "measured_in_this_run": False, "note": VALU_NOTE}
    if rank == 0 and not a.no_cpu_baseline:
        m = min(n, baseline_sample_blobs())  # bounded sample: the first blobs of this workload
        cb, dg, sums = cpu_baseline_metainfo(lens[:m], ids[:m], P, a.cpu_seconds)
        ok = all(bytes(dg[k]) == bytes(dg_h[32 * k:32 * k + 32]) for k in range(m))
        s, off = sums
        for k in range(m):
            o, cnt = int(arena.sums_off[k]), int(off[k + 1] - off[k])
            ok = ok and np.array_equal(s[int(off[k]):int(off[k + 1])], sums_h[o:o + cnt])
        cb["outputs_match_gpu"] = bool(ok)
        res["cpu_baseline"] = cb


def host_offload_leg(a, D, T, step, lens, world, dg_h, n):
    """The same batch with the library's default, krk_set_sha_host_offload(KRK_OFFLOAD_AUTO):
    the planner's longest SHA-256 chains on host threads (x86 SHA extensions, read out of
    HBM; as many threads as the process's CPU budget), the rest and every piece CRC on the
    GPU.  Reported beside `value` (which stays the GPU-only path): it is what a chain-bound
    batch (C1's one 1 GiB blob, the log-uniform regen batch) gets from the library."""
    thr = host_cores()
    idx, g_s, h_s = D.sha_offload_plan(lens, thr)
    t_idx, t_start, t_end, t_gpu = D.sha_tail_plan(lens, thr)
    gpu_only = dg_h.copy()  # step() gathers the digests into dg_h
    D.set_sha_host_offload(-1)
    try:
        for _ in range(a.warmup):
            step()
        T.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        T.barrier()
        el = T.max_over_ranks(time.perf_counter() - t0)
        tail = D.sha_last_tail()
    finally:
        D.set_sha_host_offload(0)
    total = int(sum(lens))
    if tail["chains"]:  # the run handed chain tails over (tail_plan beat whole blobs)
        on_host, host_bytes = tail["chains"], int(total - tail["gpu_prefix_bytes"] -
                                                  sum(int(lens[i]) for i in set(range(n)) - set(t_idx.tolist())))
    else:
        on_host, host_bytes = int(idx.size), int(sum(int(lens[i]) for i in idx))
    return {"value": round(world * total * a.steps / el / 1e9, 3), "unit": "GB/s",
            "ms_per_step": round(el / a.steps * 1e3, 3), "host_threads": thr, "blobs_on_host": on_host,
            "bytes_on_host": host_bytes, "blobs": n,
            "model_s": {"gpu": round(g_s, 3), "host": round(h_s, 3), "tail_handoff_end": round(t_end, 3),
                        "gpu_alone": round(t_gpu, 3)},
            "tail_handoff": {"chains": tail["chains"], "gpu_prefix_bytes": tail["gpu_prefix_bytes"]},
            "digests_match_gpu_only": bool(np.array_equal(dg_h, gpu_only)),
            "what": "krk_metainfo_digest_dev with the default offload (AUTO, host cores): whole blobs hashed on "
                    "host threads from HBM through pinned double buffers, or -- when the model ends the batch "
                    "sooner that way -- every chain started on the GPU and the longest chains' tails finished "
                    "on host threads from the GPU's midstate (tail handoff); the GPU hashes the rest and every "
                    "blob's piece CRCs (DESIGN.md 4.2)"}


def run_regen(a, D, T, rank, world, res):
    """C5 regen = Generator.Generate over a batch (lib/metainfogen/generator.go:41-58):
    NewMetaInfo per blob = piece sums on the GPU + InfoHash (bencode + SHA-1) on the
    host, batched; Generate computes no digest (core/metainfo.go:53-55 assumes it)."""
    from kraken_amd import core
    ids, lens, P = workload_blobs(a.workload, rank, world, a.blobs)
    n = len(lens)
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    pin_s = D.PinnedArray((max(arena.total_pieces, 1),), np.uint32)
    names = [f"{mix64(int(i)):016x}" * 4 for i in ids]  # the blobs' digest names (Generate takes them as given)
    packed = D.pack_names(names)
    ihs, raw = [], {}

    def step():
        if a.regen_serial:  # the unpipelined composition: all sums, then all InfoHashes
            D.piece_sums(arena, out)
            D.synchronize()
            pin_s.fill_from(out.sums)
            ihs[:] = core._info_hash_batch([P] * n, pin_s.a, arena.sums_off, arena.n_pieces, names, lens)
        else:  # krk_metainfo_batch_dev: InfoHashes of each group while the next groups' CRC runs
            # (the raw (n, 20) array, as a cgo caller gets it; Python objects are built after timing)
            raw["ih"] = D.metainfo_batch(arena, out, packed, pin_s.a)

    for _ in range(a.warmup):
        step()
    T.barrier()
    with D.KernelTimer():
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        T.barrier()
        t1 = time.perf_counter()
        crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
    if "ih" in raw:
        ihs[:] = [core.InfoHash(bytes(r)) for r in raw["ih"]]
    elapsed = T.timed_region(t1 - t0)
    bytes_rank = int(sum(lens))
    crc_avg = crc_ms / max(crc_n, 1)
    per_step = max(1, round(crc_n / max(a.steps, 1)))
    per_launch = bytes_rank / per_step
    traffic = load_traffic(a.pmc_json, a.workload, n).get("crc32_pieces")
    res.update({"metric": "metainfo regen GB/s (C5: Generator.Generate = piece sums + InfoHash per blob)",
                "value": round(world * bytes_rank * a.steps / elapsed / 1e9, 3), "unit": "GB/s", "steps": a.steps,
                "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
                "dtype": "u8", "data": "synthetic (device-generated splitmix64 blobs)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "blobs_per_gpu": n, "bytes_per_gpu": bytes_rank,
                           "piece_length": P, "pieces_per_gpu": arena.total_pieces, "mode": "device-resident"},
                "roofline": roofline_obj("crc32_pieces", per_launch / (crc_avg / 1e3) / 1e9, crc_avg, per_launch,
                                         None if traffic is None else traffic / per_step),
                "kernels": {"crc32_pieces": {"launches": crc_n, "avg_ms": round(crc_avg, 3),
                                             "launches_per_step": per_step}}})
    if per_step > 1:
        res["roofline"]["note"] = (f"the batch runs as {per_step} CRC launches a step (krk_metainfo_batch_dev "
                                   "groups); achieved = bytes per launch / average launch time; traffic = the "
                                   "single-launch PMC pass's bytes / launches per step")
    # spot-check the InfoHashes of the first blobs against the oracle's independent bencode + SHA-1
    if rank == 0:
        from oracle import oracle as O  # the checker (test infrastructure)
        O.build()
        ok = True
        for k in range(min(n, 8)):
            o, c = int(arena.sums_off[k]), int(arena.n_pieces[k])
            ok = ok and bytes(ihs[k]) == O.info_hash(P, pin_s.a[o:o + c], names[k], lens[k])
        res["info_hash_matches_oracle"] = bool(ok)
    if a.workload == "c5regen" and not a.no_e2e:
        res["end_to_end"] = regen_end_to_end(D, T, lens, P, names, world, rank, cpu=not a.no_cpu_baseline)
    if rank == 0 and not a.no_cpu_baseline:
        m = min(n, baseline_sample_blobs())
        cb, _, sums = cpu_baseline_metainfo(lens[:m], ids[:m], P, a.cpu_seconds, passes=2)
        s_, off = sums
        ok = all(np.array_equal(s_[int(off[k]):int(off[k + 1])],
                                pin_s.a[int(arena.sums_off[k]):int(arena.sums_off[k]) + int(off[k + 1] - off[k])])
                 for k in range(m))
        cb["outputs_match_gpu"] = bool(ok)
        cb["sample"] += " (the CPU side times the CRC pass only; its InfoHash is not counted)"
        res["cpu_baseline"] = cb


def run_verify(a, D, T, rank, world, res):
    """krk_verify_pieces_host over received pieces in host memory
    (the h.Sum32() != GetPieceSum(pi) check of writePiece, batched).  Inputs are
    host-resident by definition of this path, so `value` includes the PCIe pass.  The
    pieces sit in pinned receive buffers (krk_host_alloc, as INTEGRATION.md has the agent
    allocate them): the library splits the batch between host PCLMUL threads and DMA
    into the GPU by the measured rates.  `pageable` repeats it from ordinary memory
    (there the GPU side would cost a host copy per byte, so the split keeps it on the
    host unless a core copies faster than it CRCs)."""
    import ctypes as C
    from kraken_amd import agentstorage
    n, P = a.blobs or 4096, 4 << 20
    ids = [(3 << 40) + rank * n + i for i in range(n)]
    arena = D.BlobArena([P] * n, P, blob_ids=ids)  # device-generated piece content
    out = D.BatchOutputs(arena)
    D.piece_sums(arena, out)
    D.synchronize()
    expected = out.sums.to_host(np.uint32, n).copy()
    pin = D.PinnedArray((n * P,), np.uint8)
    host = pin.a
    for i in range(n):
        D.check(D.lib.krk_memcpy_d2h(C.c_void_p(host.ctypes.data + i * P), arena.buf.ptr + int(arena.offsets[i]), P))
    del out, arena
    datas = [host[i * P:(i + 1) * P] for i in range(n)]
    want = np.ones(n, dtype=bool)
    want[::64] = False
    exp = expected.copy()
    exp[~want] ^= 0x5A5A5A5A  # corrupted pieces: GetPieceSum disagrees with the bytes
    got = [None]

    def step():
        got[0] = agentstorage.verify_pieces(datas, exp)

    for _ in range(a.warmup):
        step()
    T.barrier()
    with D.KernelTimer():
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        T.barrier()
        t1 = time.perf_counter()
        crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
    elapsed = T.timed_region(t1 - t0)
    bytes_rank = n * P
    rates = D.planner_rates()
    g_bytes, h_bytes, frac_next = D.crc_host_split()  # the last step's split
    per_launch = g_bytes * a.steps / max(crc_n, 1)
    crc_avg = crc_ms / max(crc_n, 1)
    roof = roofline_obj("crc32_pieces", per_launch / (crc_avg / 1e3) / 1e9 if crc_n else 0.0, crc_avg, per_launch,
                        None)
    roof["note"] = ("achieved = the GPU's share of a step's bytes (split.gpu_bytes) per launch / average launch time; "
                    "that share goes up by DMA in pinned windows, one CRC launch per window, so the call is bounded "
                    "by the host link and the host threads' PCLMUL rate, not by the kernel")
    if not crc_n:  # the split measured host-only faster: the host threads are the whole call
        cap = host_cores() * rates["host_crc_bps"] / 1e9
        v = world * bytes_rank * a.steps / elapsed / 1e9
        roof = {"kernel": None, "bound": "host PCLMUL threads", "achieved": round(v, 3), "peak": round(cap, 3),
                "unit": "GB/s", "frac": round(v / cap, 4) if cap else None, "traffic": None,
                "note": "no byte went to the GPU in the timed steps (the learned split measured host-only faster, "
                        "DESIGN.md 4.5); peak = the CPU budget's threads x one thread's measured PCLMUL rate"}
    res.update({"metric": "agent piece-verify GB/s (host pieces, end to end)",
                "value": round(world * bytes_rank * a.steps / elapsed / 1e9, 3), "unit": "GB/s", "steps": a.steps,
                "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
                "dtype": "u8", "data": "synthetic (device-generated splitmix64 pieces, copied to pinned host memory)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "pieces_per_gpu": n, "piece_length": P,
                           "bytes_per_gpu": bytes_rank, "mode": "host buffers (pinned receive buffers), "
                                                                 "host threads + GPU by measured rates"},
                "roofline": roof, "kernels": {"crc32_pieces": {"launches": crc_n, "avg_ms": round(crc_avg, 3)}},
                "planner_rates": {k: (round(v / 1e9, 3) if isinstance(v, float) else v) for k, v in rates.items()
                                  if k != "sha_stream_bps"},
                "split": {"gpu_bytes": g_bytes, "host_bytes": h_bytes, "gpu_share_next": round(frac_next, 4),
                          "host_threads": host_cores(),
                          "what": "the last step's bytes on the GPU (DMA from the pinned pieces) and on host PCLMUL "
                                  "threads; the share is learned from the measured rates of both sides"},
                "verdicts_match": bool(np.array_equal(got[0], want))})
    if world == 1 and not a.no_cpu_baseline:
        res["same_buffer"] = same_buffer_ab(step, [host.ctypes.data + i * P for i in range(n)], [P] * n, expected)
    # the same pieces from pageable memory
    pg = np.empty(n * P, dtype=np.uint8)
    pg[:] = host
    pdatas = [pg[i * P:(i + 1) * P] for i in range(n)]
    pv = agentstorage.verify_pieces(pdatas, exp)
    T.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pv = agentstorage.verify_pieces(pdatas, exp)
    T.barrier()
    el = T.max_over_ranks(time.perf_counter() - t0)
    res["pageable"] = {"value": round(world * bytes_rank * a.steps / el / 1e9, 3), "unit": "GB/s",
                       "verdicts_match": bool(np.array_equal(pv, want)),
                       "what": "the same batch from pageable host memory (numpy)"}
    del pg, pdatas
    if rank == 0 and not a.no_cpu_baseline:
        # 512 pieces = 2 GiB of distinct bytes: a sample of a few hundred MiB would sit in the
        # host's last-level cache across the repeated passes and overstate the CPU rate
        m = min(n, 512)
        cb, _, sums = cpu_baseline_metainfo([P] * m, ids[:m], P, a.cpu_seconds, passes=2)
        s_, off = sums
        cb["outputs_match_gpu"] = bool(np.array_equal(np.asarray(s_[:m], dtype=np.uint32), expected[:m]))
        cb["sample"] += " (one CRC per piece: the reference's hash.Hash32 per received piece)"
        if "same_buffer" in res:  # like for like -- the oracle over the very pieces verified
            res["cpu_baseline_own_sample"] = cb
            res["cpu_baseline"] = same_buffer_baseline(res["same_buffer"], n, P, "pinned receive pieces")
        else:
            res["cpu_baseline"] = cb


def host_mem_budget():
    """Bytes of host memory this process may use: physical memory or the cgroup limit,
    whichever is lower."""
    try:
        phys = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    except (ValueError, OSError):
        phys = 1 << 40
    for f in ("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory/memory.limit_in_bytes"):
        try:
            v = open(f).read().strip()
            if v.isdigit():
                phys = min(phys, int(v))
        except OSError:
            pass
    return phys


E2E_PASSES = 3


_LINK_PEAK = {}


def host_link_peak(D):
    """One GPU's host link, GB/s: the best of five 256 MiB pinned host-to-device copies timed
    here (once a process), or the planner's calibration figure (one 64 MiB copy at krk_init,
    krk_planner_rates_get) when that is higher.  The single calibration copy alone can read
    low -- 45.7 against ~56 GB/s on one box, which put an end-to-end pass at 1.11 of "the
    link" -- so the roofline takes the larger of the two."""
    if "GBps" not in _LINK_PEAK:
        import ctypes as C
        nb = 256 << 20
        h = D.PinnedArray((nb,), np.uint8, dma_target=True)
        d = D.DeviceBuffer(nb)
        best = 0.0
        try:
            h.a[:] = 1
            for rep in range(6):  # the first copy warms the path and is not counted
                t0 = time.perf_counter()
                D.check(D.lib.krk_memcpy_h2d(C.c_void_p(d.ptr), C.c_void_p(h.ptr), nb))
                dt = time.perf_counter() - t0
                if rep:
                    best = max(best, nb / dt / 1e9)
        finally:
            d.free()
        planner = D.planner_rates()["h2d_bps"] / 1e9
        _LINK_PEAK.update({"GBps": max(best, planner), "measured_GBps": round(best, 3),
                           "planner_GBps": round(planner, 3)})
    return _LINK_PEAK


def link_roofline(D, gbps, traffic_workload=None, n=None, world=1):
    """An end-to-end pass is bounded by the host link: every byte crosses PCIe once.  Peak =
    one GPU's pinned H2D rate (host_link_peak) x the ranks (`gbps` is the whole job's).  With
    `traffic_workload`, the kernels' HBM bytes per window launch from the committed PMC
    passes of that leg (tools/pmc_traffic.py) ride along: the windows' kernels read each
    staged byte once (traffic over the 512 MiB window ~1.00)."""
    lp = host_link_peak(D)
    h2d = lp["GBps"] * max(1, int(world))
    r = {"bound": "host link (PCIe H2D)", "achieved": round(gbps, 3), "peak": round(h2d, 3), "unit": "GB/s",
         "frac": round(gbps / h2d, 4) if h2d else None,
         "peak_source": f"pinned H2D per GPU x {max(1, int(world))} rank(s): the larger of the best of five 256 MiB "
                        f"copies timed in this run ({lp['measured_GBps']}) and the planner's calibration copy "
                        f"({lp['planner_GBps']}, krk_planner_rates_get)", "traffic": None}
    if traffic_workload:
        t = load_traffic(None, traffic_workload, n)
        if t:
            win = window_bytes_default()
            r["traffic"] = {"per_window_launch": {k: t[k] for k in ("crc32_pieces", "sha256_multi") if k in t},
                            "window_bytes": win,
                            "over_algorithmic": {k: round(t[k] / win, 4) for k in ("crc32_pieces", "sha256_multi")
                                                 if k in t},
                            "source": f"{TRAFFIC_FOUND.get(traffic_workload)} (FETCH_SIZE/WRITE_SIZE "
                                      "passes, gfx950 correction)"}
    return r


def window_bytes_default():
    """Bytes of one staging window (KRK_WINDOW_MB, default 512 MiB: staging.hpp window_bytes)."""
    return int(os.environ.get("KRK_WINDOW_MB", "512")) << 20


def host_sources(D, k, nbytes, seed):
    """k sources of `nbytes` device-generated (splitmix64) bytes, copied to pageable host
    arrays: the end-to-end legs' blobs are prefixes of them (distinct bytes well above the
    host's caches, without holding every blob's bytes)."""
    out = []
    buf = D.DeviceBuffer(nbytes)
    try:
        for s in range(k):
            D.check(D.lib.krk_synth_fill_dev(buf.ptr, seed + s, 0, nbytes, 0, None))
            D.synchronize()
            out.append(buf.to_host(np.uint8, nbytes))
    finally:
        buf.free()
    return out


def timed_passes(T, fn, passes=3):
    """Median over `passes` runs of fn() (each bracketed by barriers, max over ranks) and the
    last run's result."""
    ts, r = [], None
    for _ in range(passes):
        T.barrier()
        t0 = time.perf_counter()
        r = fn()
        ts.append(T.max_over_ranks(time.perf_counter() - t0))
    return float(np.median(ts)), ts, r


def host_crc_ceiling(D):
    """What the host side of a CRC-only host-resident call can reach: the host's PCLMUL
    capacity (threads x one thread's measured rate) and the host link (pinned H2D)."""
    R = D.planner_rates()
    return {"host_crc_GBps": round(host_cores() * R["host_crc_bps"] / 1e9, 2), "threads": host_cores(),
            "host_crc_GBps_per_thread": round(R["host_crc_bps"] / 1e9, 3), "h2d_GBps": round(R["h2d_bps"] / 1e9, 2),
            "source": "krk_planner_rates_get (measured on this box at krk_init)"}


def same_buffer_ab(lib_pass, ptrs, lens, want, rounds=3):
    """The library's host pass and the oracle's per-piece CRC (orc_crc_bufs: the reference's
    crc32 per piece, every host core taking pieces in turn) over the SAME host bytes,
    alternated `rounds` times: host-memory bandwidth on these boxes moves by 2x between
    minutes (placement, the host's other tenants), so a baseline timed on its own sample at
    another moment is no like-for-like.  Medians; the oracle's sums are checked against
    `want`."""
    from oracle import oracle as O  # the CPU baseline leg (test infrastructure)
    O.build()
    total = float(sum(int(x) for x in lens))
    lib_t, orc_t, ok = [], [], True
    for _ in range(rounds):
        t0 = time.perf_counter()
        lib_pass()
        lib_t.append(time.perf_counter() - t0)
        t, sums = O.crc_bufs(ptrs, lens, node_cores())
        orc_t.append(t)
        ok = ok and bool(np.array_equal(sums, want))
    med = lambda v: sorted(v)[len(v) // 2]
    return {"library_GBps": round(total / med(lib_t) / 1e9, 3), "oracle_GBps": round(total / med(orc_t) / 1e9, 3),
            "library_s": [round(x, 4) for x in lib_t], "oracle_s": [round(x, 4) for x in orc_t],
            "oracle_threads": node_cores(), "oracle_sums_match": ok,
            "what": "library pass and oracle pass (crc32 per piece on every host core, oracle/oracle.c orc_crc_bufs) "
                    f"alternated {rounds}x over the same host buffer; medians"}


def same_buffer_baseline(sb, k, P, what):
    """The cpu_baseline of a host-resident CRC leg: the reference
    verifies pieces in the buffers it received them into (lib/torrent/storage/agentstorage/
    torrent.go:175-199), so the baseline is the oracle's pass over the SAME bytes the library
    just read, alternated with it (same_buffer_ab), not its own first-touched sample."""
    return {"value": sb["oracle_GBps"], "unit": "GB/s", "cores": sb["oracle_threads"], "cores_source": CORES_SOURCE,
            "kind": "port",
            "sample": (f"the same {k} {what} of {P >> 10} KiB ({k * P / 2**30:.1f} GiB) the library read, alternated "
                       f"with its pass {len(sb['oracle_s'])}x (median): crc32 per piece on every host core, "
                       "oracle/oracle.c orc_crc_bufs"),
            "outputs_match_gpu": sb["oracle_sums_match"], "library_same_buffer_GBps": sb["library_GBps"]}


def c4_end_to_end(D, T, arena, want_sums, P, world, ab=False):
    """C4's blob in HOST memory (VERDICT r03 missing #2): krk_piece_sums_host over the 20 GiB
    blob in a pinned receive buffer (the library splits whole pieces between host PCLMUL
    threads and DMA into the GPU by the measured rates) and in pageable memory (host
    threads: a staging copy per byte would cost more than the GPU saves).  Sums equal the
    device-resident run's."""
    import ctypes as C
    L = int(arena.lengths[0])
    per_rank = 0.4 * host_mem_budget() / max(1, world)
    if world > 1:
        per_rank = min(per_rank, 24 << 30)
    Le = min(L, int(per_rank / 2) // P * P)
    pin = D.PinnedArray((Le,), np.uint8)
    D.check(D.lib.krk_memcpy_d2h(C.c_void_p(pin.a.ctypes.data), arena.buf.ptr + int(arena.offsets[0]), Le))
    pg = np.empty(Le, dtype=np.uint8)
    pg[:] = pin.a
    k = Le // P
    res = {"unit": "GB/s", "blob_bytes": Le, "piece_length": P,
           **({"blob_bytes_requested": L, "capped_by": "host memory per rank"} if Le < L else {}),
           "ceiling": host_crc_ceiling(D)}
    for name, buf in (("pinned", pin.a), ("pageable", pg)):
        for _ in range(3):  # warm: two pinned calls split (the first sets up), one runs host-only, then the faster
            D.piece_sums_host([buf], P)
        el, ts, r = timed_passes(T, lambda: D.piece_sums_host([buf], P))
        g, h, frac = D.crc_host_split()
        res[name] = {"value": round(world * Le / el / 1e9, 3), "seconds": round(el, 3),
                     "passes_s": [round(x, 3) for x in ts], "gpu_bytes": g, "host_bytes": h,
                     "sums_match_device_run": bool(np.array_equal(r[0][:k], want_sums[:k]))}
    if ab:  # rank 0 at N=1: the reference's per-piece CRC over the same pinned bytes, alternated
        base = pin.a.ctypes.data
        res["pinned"]["same_buffer"] = same_buffer_ab(lambda: D.piece_sums_host([pin.a], P),
                                                      [base + i * P for i in range(k)], [P] * k, want_sums[:k])
        res["pinned"]["same_buffer"]["what"] += (" (generous to the reference: its calcPieceSums is one goroutine "
                                                 "per blob, cpu_baseline.one_goroutine)")
        res["cpu_baseline"] = same_buffer_baseline(res["pinned"]["same_buffer"], k, P, "pieces of the pinned blob")
    res["value"] = res["pinned"]["value"]
    res["what"] = ("the blob in host memory through krk_piece_sums_host (agent verify / Generate over a host "
                   "buffer): `pinned` = a krk_host_alloc receive buffer (host threads + GPU DMA by the measured "
                   "rates), `pageable` = ordinary memory (host threads); median of 3 passes")
    del pin, pg
    return res


def regen_end_to_end(D, T, lens, P, names, world, rank, cpu=True):
    """C5 regen from the CAS files themselves (VERDICT r03 missing #2): Generate over cache
    files = krk_piece_sums_files + the InfoHash batch, on the library's default CRC placement
    (AUTO: the measured crossover; HOST on a box whose PCLMUL capacity exceeds the link) and
    forced onto the GPU (files -> pinned windows -> PCIe -> CRC kernel), and from pageable
    host memory (krk_piece_sums_host).  Blob i = a prefix of one of 4 source files (4 GiB of
    distinct bytes, page cache warm after the first pass).  The placements' sums are equal;
    three blobs (shortest, median, longest) equal the oracle."""
    import shutil
    import tempfile
    from kraken_amd import core
    n, K = len(lens), 4
    top = max(lens)
    srcs = host_sources(D, K, top, (6 << 40) + rank * K)
    d = tempfile.mkdtemp(prefix=f"krk_regen_r{rank}_")
    try:
        for k, x in enumerate(srcs):
            with open(os.path.join(d, f"src{k}"), "wb") as f:
                f.write(memoryview(x))
        paths = [os.path.join(d, f"src{i % K}") for i in range(n)]
        counts = np.asarray([int(D.lib.krk_num_pieces(L, P)) for L in lens], dtype=np.uint64)
        total = int(sum(lens))

        def gen_files():
            sums, offs = D.piece_sums_files(paths, lens, P)
            return sums, core._info_hash_batch([P] * n, sums, offs[:-1], counts, names, lens)

        legs = {}
        for name, place in (("default", D.PLACE_AUTO), ("gpu", D.PLACE_GPU)):
            D.set_crc_placement(place)
            try:
                gen_files()  # warm (page cache, staging windows)
                el, ts, r = timed_passes(T, gen_files)
                g, h, _ = D.crc_host_split()
            finally:
                D.set_crc_placement(D.PLACE_AUTO)
            legs[name] = {"value": round(world * total / el / 1e9, 3), "seconds": round(el, 3),
                          "passes_s": [round(x, 3) for x in ts], "placement": "gpu" if g else "host", "result": r}
        datas = [srcs[i % K][:lens[i]] for i in range(n)]

        def gen_mem():
            per = D.piece_sums_host(datas, P)
            sums = np.concatenate(per) if per else np.zeros(0, np.uint32)
            offs = np.zeros(n + 1, dtype=np.uint64)
            offs[1:] = np.cumsum(counts)
            return sums, core._info_hash_batch([P] * n, sums, offs[:-1], counts, names, lens)

        gen_mem()
        el_m, ts_m, r_m = timed_passes(T, gen_mem)
        cpu_files = None
        if cpu and rank == 0:  # the reference's own Generate over the same files on the CPU budget
            from oracle import oracle as O  # the CPU baseline leg (test infrastructure)
            O.build()
            # library and oracle alternated over the same files (host memory bandwidth on these
            # boxes moves by 2x between minutes, so separate passes are no like-for-like)
            runs, t_lib = [], []
            D.set_crc_placement(D.PLACE_AUTO)
            for _ in range(3):
                t0 = time.perf_counter()
                gen_files()
                t_lib.append(time.perf_counter() - t0)
                runs.append(O.baseline_files(paths, lens, P, node_cores()))
            t_c = float(np.median([r[0] for r in runs]))
            cpu_files = {"value": round(total / t_c / 1e9, 3), "unit": "GB/s", "cores": node_cores(),
                         "cores_source": CORES_SOURCE, "kind": "port",
                         "seconds": round(t_c, 3),
                         "library_alternated_GBps": round(total / float(np.median(t_lib)) / 1e9, 3),
                         "library_alternated_s": [round(x, 3) for x in t_lib],
                         "oracle_s": [round(r[0], 3) for r in runs],
                         "sums_match": bool(np.array_equal(runs[0][1][:int(counts.sum())],
                                                           legs["default"]["result"][0][:int(counts.sum())])),
                         "sample": "the same 1,000 files (page cache warm): calcPieceSums over each file reader, "
                                   "32 KiB reads folded with PCLMUL, one file per thread (oracle/oracle.c "
                                   "orc_baseline_files), alternated 3x with the library's default pass "
                                   "(library_alternated_GBps, InfoHash included there); median of 3; InfoHash "
                                   "not counted on the oracle's side"}
        same = all(np.array_equal(legs["default"]["result"][0][:int(counts.sum())], x[0][:int(counts.sum())])
                   and list(legs["default"]["result"][1]) == list(x[1]) for x in (legs["gpu"]["result"], r_m))
        from oracle import oracle as O  # checker only
        O.build()
        L = np.asarray(lens)
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(counts)
        ok = True
        for i in sorted({int(L.argmin()), int(np.argsort(L)[n // 2]), int(L.argmax())}):
            got = legs["default"]["result"][0][int(offs[i]):int(offs[i + 1])]
            ok = ok and np.array_equal(got, O.calc_piece_sums(srcs[i % K][:lens[i]], P)[1])
    finally:
        shutil.rmtree(d, ignore_errors=True)
    for v in legs.values():
        v.pop("result")
    legs["gpu"]["roofline"] = link_roofline(D, legs["gpu"]["value"], world=world)
    return {"value": legs["default"]["value"], "unit": "GB/s", "blobs": n, "bytes": total,
            "files": legs, "pageable_memory": {"value": round(world * total / el_m / 1e9, 3),
                                               "seconds": round(el_m, 3), "passes_s": [round(x, 3) for x in ts_m]},
            "ceiling": host_crc_ceiling(D), "cpu_baseline_files": cpu_files,
            "outputs_equal_across_paths": bool(same),
            "oracle_sampled_match": bool(ok),
            "what": "Generator.Generate over cache files (piece sums + InfoHash batch): `files.default` on the "
                    "library's default CRC placement, `files.gpu` forced through the pinned windows and the CRC "
                    "kernel, `pageable_memory` over host buffers; median of 3 passes"}


def c3_end_to_end(D, T, world, rank):
    """C3's length law / 64 (16,384 blobs of 1.6-16.8 MB, 151 GB) from PAGEABLE host memory
    through krk_metainfo_digest_host (VERDICT r03 missing #2: C3's device-generated figure
    is no caller's rate; real bytes cross the host link): GPU only, and the library's default
    (AUTO host offload).  Blob i = a prefix of one of 64 sources.  The files and pinned
    forms of the same law are `bench.py --workload files`."""
    n, SRC, P = 16384, 64, 4 << 20
    lens = c3_lengths(n, scale=64)
    srcs = host_sources(D, SRC, max(lens), (3 << 40) + rank * SRC)
    datas = [srcs[i % SRC][:lens[i]] for i in range(n)]
    total = int(sum(lens))
    D.set_sha_host_offload(0)
    D.metainfo_digest_host(datas, P)  # warm
    el, ts, (sums, dg) = timed_passes(T, lambda: D.metainfo_digest_host(datas, P), passes=2)
    st = D.windows_last_call()
    D.set_sha_host_offload(-1)
    try:
        el_a, ts_a, (sums_a, dg_a) = timed_passes(T, lambda: D.metainfo_digest_host(datas, P), passes=2)
        st_a = D.windows_last_call()
    finally:
        D.set_sha_host_offload(0)
    same = bool(np.array_equal(dg, dg_a)) and all(np.array_equal(x, y) for x, y in zip(sums, sums_a))
    import hashlib
    L = np.asarray(lens)
    ok = all(bytes(dg[i]) == hashlib.sha256(srcs[i % SRC][:lens[i]].tobytes()).digest()
             for i in sorted({int(L.argmin()), int(L.argmax())}))
    full = int(sum(c3_lengths(20000)))
    v = world * total / el / 1e9
    return {"value": round(v, 3), "unit": "GB/s", "blobs": n, "bytes": total, "seconds": round(el, 3),
            "passes_s": [round(x, 3) for x in ts], "windows": st, "roofline": link_roofline(D, v, world=world),
            "default_offload": {"value": round(world * total / el_a / 1e9, 3), "passes_s": [round(x, 3) for x in ts_a],
                                "host_blobs": st_a["host_blobs"]},
            "outputs_equal_across_paths": same, "digests_sampled_match_hashlib": bool(ok),
            "projected_full_c3_s": round(full / (v * 1e9), 1),
            "what": "the C3 law / 64 from pageable host memory, GPU only (host offload off) and the library's default; "
                    "projected_full_c3_s = C3's 11.7 TB at this rate across the job's host links"}


def end_to_end(D, T, arena, n, Le, P, out, world):
    """End-to-end leg (reported beside `value`, never as it): the same blobs' first
    Le bytes in pageable host memory, through krk_metainfo_digest_host (pinned
    windows, one PCIe pass feeding both kernels), results back on the host.  Every
    rank holds n * Le bytes of host memory at once, so with several ranks per node the
    bytes per blob are capped to 40 % of the host memory over the ranks (reported)."""
    import ctypes as C
    want = Le
    # host memory per rank: 40 % of the host's over the ranks, and at most 24 GiB a rank when
    # several ranks share the node (8 ranks x 100 GB of pageable copies would crowd the host)
    per_rank = 0.4 * host_mem_budget() / max(1, world)
    if world > 1:
        per_rank = min(per_rank, 24 << 30)
    cap = int(per_rank / max(1, n)) // P * P
    if cap < Le:
        Le = max(P, cap)
    datas = [np.empty(Le, dtype=np.uint8) for _ in range(n)]
    for i, d in enumerate(datas):  # the device blobs' prefixes (device-generated content)
        D.check(D.lib.krk_memcpy_d2h(d.ctypes.data_as(C.c_void_p), arena.buf.ptr + int(arena.offsets[i]), Le))
    D.metainfo_digest_host([d[:1 << 20] for d in datas[:2]], P)  # warm the staging windows (short chains)
    paths = {}
    # the staged path (pageable -> pinned window copies on host threads,
    # then the DMA: three host-DRAM touches a byte) against the gather (the pages registered,
    # each window read over PCIe by one gather launch: one touch), same batch, same box
    # (the A/B at N=1; N>1 lines run the default path only: 8 ranks registering their batches
    # at once is an experiment, not the library's default)
    for name, mode in ((("staged", 0), ("gather", 1)) if world == 1 else (("staged", 0),)):
        D.set_host_gather(mode)
        passes, cpu = [], []
        try:
            for _ in range(E2E_PASSES):  # the host side of a box varies pass to pass: the median is reported
                T.barrier()
                c0, t0 = cpu_seconds(), time.perf_counter()
                sums, dg = D.metainfo_digest_host(datas, P)
                cpu.append(cpu_seconds() - c0)
                passes.append(T.max_over_ranks(time.perf_counter() - t0))
            st = D.windows_last_call()
        finally:
            D.set_host_gather(-1)
        el_p = float(np.median(passes))
        gbps = world * n * Le / el_p / 1e9
        paths[name] = {"GBps": round(gbps, 3), "passes_s": [round(x, 3) for x in passes],
                       "host_cpu_s_per_GB": round(float(np.median(cpu)) / (n * Le / 1e9), 4),
                       "h2d_frac": None, "windows": st["windows"], "gather_windows": st["gather_windows"],
                       "registered_bytes": st["registered_bytes"], "register_s": round(st["register_s"], 3)}
        paths[name]["_sums_dg"] = (sums, dg)
    h2d = host_link_peak(D)["GBps"]
    for v in paths.values():
        v["h2d_frac"] = round(v["GBps"] / world / h2d, 4) if h2d else None
    best = max(paths, key=lambda k: paths[k]["GBps"])
    same_paths = None
    if "gather" in paths:
        same_paths = bool(np.array_equal(paths["staged"]["_sums_dg"][1], paths["gather"]["_sums_dg"][1]) and all(
            np.array_equal(a, b) for a, b in zip(paths["staged"]["_sums_dg"][0], paths["gather"]["_sums_dg"][0])))
    sums, dg = paths[DEFAULT_HOST_PATH]["_sums_dg"]
    for v in paths.values():
        del v["_sums_dg"]
    el = world * n * Le / (paths[DEFAULT_HOST_PATH]["GBps"] * 1e9)
    passes = paths[DEFAULT_HOST_PATH]["passes_s"]
    k = Le // P
    ok = None
    if out is not None and k:
        dev_sums = out.sums.to_host(np.uint32, arena.total_pieces)
        ok = all(np.array_equal(sums[i][:k], dev_sums[int(arena.sums_off[i]):int(arena.sums_off[i]) + k])
                 for i in range(n))
    res = {"value": round(world * n * Le / el / 1e9, 3), "unit": "GB/s", "blobs_per_gpu": n, "blob_bytes": Le,
           **({"blob_bytes_requested": want, "capped_by": "host memory per rank (40 % / ranks, <= 24 GiB with "
                                                          "several ranks)"} if Le < want else {}),
           "seconds": round(el, 3), "passes_s": [round(x, 3) for x in passes],
           "source": f"pageable host memory (numpy), the library's default path ({DEFAULT_HOST_PATH}); median of "
                     "the passes",
           "paths": paths, "faster_path": best, "paths_outputs_equal": same_paths,
           "bound": "PCIe H2D (one pass per byte) and the per-blob SHA-256 chain (blob_bytes / per-stream rate)",
           "sums_match_device_run": ok,
           "roofline": link_roofline(D, world * n * Le / el / 1e9, "c2_end_to_end", n, world=world)}
    if out is not None and Le == int(arena.lengths[0]) and (arena.lengths == Le).all():  # whole blobs
        dev_dg = out.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
        res["digests_match_device_run"] = bool(np.array_equal(dg, dev_dg))
    hyb = [host_hybrid(D, T, datas, P, thr, sums, dg, world) for thr in E2E_HYBRID_THREADS]
    if hyb:
        res["host_hybrid"] = hyb[0] if len(hyb) == 1 else hyb
    del datas
    return res


# The library's default for a pageable host batch (krk_set_host_gather AUTO): the staging
# copy -- measured faster than registering the caller's 4 KiB pages for the gather (VERDICT
# r04 item 3); the leg measures both and reports which was faster.
DEFAULT_HOST_PATH = "staged"


def cpu_seconds() -> float:
    """This process's user + system CPU seconds (every thread)."""
    import resource
    u = resource.getrusage(resource.RUSAGE_SELF)
    return u.ru_utime + u.ru_stime


# Host threads of the end-to-end leg's hybrid pass (KRK_BENCH_HYBRID="8,16"; "" = none;
# -1 = the library's default, KRK_OFFLOAD_AUTO: a quarter of the CPU budget for host-resident
# batches).
E2E_HYBRID_THREADS = [int(x) for x in os.environ.get("KRK_BENCH_HYBRID", "-1").split(",") if x.strip()]


def host_hybrid(D, T, datas, P, thr, sums_gpu, dg_gpu, world):
    """The end-to-end batch again with krk_set_sha_host_offload(thr): the planner hands the
    host the blobs the link would carry past the GPU's own chain time; those are hashed
    and piece-summed in place on host threads and never uploaded, the rest go through
    the windows as before.  Reported beside the GPU-only end-to-end figure, with the
    outputs checked equal to it."""
    lens = [int(d.size) for d in datas]
    if thr < 0:
        thr_plan = max(1, host_cores() // 4)  # what KRK_OFFLOAD_AUTO uses for host-resident batches
    else:
        thr_plan = thr
    idx, g_s, h_s = D.sha_offload_plan(lens, thr_plan, mode=D.OFFLOAD_HOST_WHOLE)
    passes = []
    D.set_sha_host_offload(thr)
    try:
        for _ in range(E2E_PASSES):
            T.barrier()
            t0 = time.perf_counter()
            sums, dg = D.metainfo_digest_host(datas, P)
            passes.append(T.max_over_ranks(time.perf_counter() - t0))
    finally:
        D.set_sha_host_offload(0)
    el = float(np.median(passes))
    same = bool(np.array_equal(dg, dg_gpu)) and all(np.array_equal(a, b) for a, b in zip(sums, sums_gpu))
    return {"threads": thr_plan, "auto": thr < 0, "value": round(world * sum(lens) / el / 1e9, 3), "unit": "GB/s",
            "seconds": round(el, 3), "passes_s": [round(x, 3) for x in passes], "blobs_on_host": int(idx.size),
            "model_s": {"gpu": round(g_s, 3), "host": round(h_s, 3)}, "outputs_match_gpu_only": same,
            "what": "krk_metainfo_digest_host with the host offload on (auto: the library's default): the planner's blobs are "
                    "hashed and piece-summed in place on host threads and never cross PCIe, the rest as in the "
                    "GPU-only pass (DESIGN.md 4.5); median of the passes"}


def run_pieces(a, D, T, rank, world, res):
    ids, lens, P = workload_blobs(a.workload, rank, world, a.blobs)
    arena = D.BlobArena(lens, P, blob_ids=ids)
    out = D.BatchOutputs(arena)
    pin_s = D.PinnedArray((max(arena.total_pieces, 1),), np.uint32)  # results gathered to pinned host memory
    sums_h = pin_s.a

    # Timed steps are serial (each step's sums on the host before the next is enqueued), so
    # every launch runs alone and its hipEvent time is the kernel's own (the roofline).
    # Then the same steps back to back (a Generator working through a queue of layers):
    # step k runs on stream k % 2 into its own sums buffer and pinned result array and is
    # enqueued before the host waits for step k - 1, so the host's enqueue (~0.2 ms:
    # descriptor upload, launch) and each launch's tail overlap the neighbouring layer's
    # kernel -- reported as `back_to_back`.
    import ctypes as C
    streams = [C.c_void_p(), C.c_void_p()]
    for st in streams:
        D.check(D.lib.krk_stream_create(C.byref(st)))
    outs = [out, D.BatchOutputs(arena)]
    pins = [pin_s, D.PinnedArray((max(arena.total_pieces, 1),), np.uint32)]

    def enqueue(k):
        D.piece_sums(arena, outs[k & 1], stream=streams[k & 1])
        pins[k & 1].fill_from_async(outs[k & 1].sums, streams[k & 1])

    def run(nsteps, serial):
        for k in range(nsteps):
            enqueue(k)
            if serial:
                D.check(D.lib.krk_stream_sync(streams[k & 1]))
            elif k:
                D.check(D.lib.krk_stream_sync(streams[(k - 1) & 1]))
        if nsteps:
            D.check(D.lib.krk_stream_sync(streams[(nsteps - 1) & 1]))

    run(a.warmup, True)
    T.barrier()
    with D.KernelTimer():
        t0 = time.perf_counter()
        run(a.steps, True)
        T.barrier()
        t1 = time.perf_counter()
        crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
    sums_h = pins[(a.steps - 1) & 1].a if a.steps else sums_h
    want = sums_h.copy()
    T.barrier()
    t2 = time.perf_counter()
    run(a.steps, False)
    T.barrier()
    el_b2b = T.max_over_ranks(time.perf_counter() - t2)
    same = all(np.array_equal(p.a, want) for p in pins)
    for st in streams:
        D.lib.krk_stream_destroy(st)
    elapsed = T.timed_region(t1 - t0)
    bytes_rank = int(sum(lens))
    crc_avg = crc_ms / max(crc_n, 1)
    crc_gbps = bytes_rank / (crc_avg / 1e3) / 1e9
    res.update({"metric": "piece-sum (NewMetaInfo CRC-32) GB/s",
                "value": round(world * bytes_rank * a.steps / elapsed / 1e9, 3), "unit": "GB/s",
                "steps": a.steps, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "dtype": "u8", "data": "synthetic (device-generated splitmix64 blobs)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "bytes_per_gpu": bytes_rank,
                           "piece_length": P, "pieces_per_gpu": arena.total_pieces, "mode": "device-resident",
                           "steps": "serial (each step's sums on the host before the next is enqueued)"},
                "back_to_back": {"value": round(world * bytes_rank * a.steps / el_b2b / 1e9, 3), "unit": "GB/s",
                                 "ms_per_step": round(el_b2b / a.steps * 1e3, 3), "sums_match_serial": same,
                                 "what": "the same steps with step k+1 enqueued while step k runs (two streams, "
                                         "two sums buffers, every step's sums in pinned host memory)"},
                "roofline": roofline_obj("crc32_pieces", crc_gbps, crc_avg, bytes_rank,
                                         load_traffic(a.pmc_json, a.workload, len(lens)).get("crc32_pieces")),
                "kernels": {"crc32_pieces": {"launches": crc_n, "avg_ms": round(crc_avg, 3)}}})
    # InfoHash over the 81,920 sums stays on the host (bencode + SHA-1, core/metainfo.go:37-44)
    from kraken_amd import core
    t0 = time.perf_counter()
    core._info_hash(P, sums_h[:arena.total_pieces], "0" * 64, lens[0])
    res["info_hash_host_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    if a.workload == "c4" and not a.no_e2e:
        res["end_to_end"] = c4_end_to_end(D, T, arena, sums_h, P, world, ab=world == 1 and not a.no_cpu_baseline)
    if rank == 0 and not a.no_cpu_baseline:
        m = 2 * node_cores()
        cb, _, sums = cpu_baseline_metainfo([256 << 20] * m, [ids[0]] * m, P, a.cpu_seconds, passes=2)
        s, off = sums
        cnt = int(off[1] - off[0])
        cb["outputs_match_gpu"] = bool(np.array_equal(s[:cnt], sums_h[:cnt]))
        cb["sample"] += (" (sample blobs: 256 MiB prefixes of the same synthetic blob, one a thread: C4's "
                         "ONE blob would be one goroutine in the reference, see one_goroutine)")
        # the reference's calcPieceSums over C4's single blob runs on one goroutine
        # (core/metainfo.go:157-179): one thread over one 256 MiB prefix
        c1, _, _ = cpu_baseline_metainfo([256 << 20], [ids[0]], P, min(a.cpu_seconds, 3.0), passes=2)
        cb["one_goroutine"] = {"value": c1["value"], "unit": "GB/s", "cores": 1,
                               "what": "the reference's calcPieceSums over the one C4 blob: a single "
                                       "goroutine (one thread, 256 MiB sample)"}
        res["cpu_baseline"] = cb


def run_chunked(a, D, T, rank, world, res):
    """C3: every blob of this rank's LPT shard advances by one chunk per window; the
    next window's bytes are generated on the device (own stream) while the current
    window's kernels run (kraken_amd.windowed, the machinery tests/test_gpu_windowed.py
    checks against the oracle)."""
    from kraken_amd.windowed import WindowedRun
    # --emulate-world W: run rank `rank`'s LPT shard of a W-GPU run on this one GPU (ranks
    # share nothing, so a W-GPU run takes as long as its slowest shard; rank 0 holds the
    # longest blob, whose chain bounds every shard).
    shard_world = a.emulate_world or world
    shard_rank = rank if a.emulate_rank is None else a.emulate_rank  # --emulate-rank: another rank's shard
    assert 0 <= shard_rank < shard_world, (shard_rank, shard_world)
    ids, lens, P = workload_blobs(a.workload, shard_rank, shard_world, a.blobs)
    n = len(lens)
    if a.c3_tail_only:  # a measurement run of the tail handoff alone (no value line)
        res.update({"metric": "C3 tail handoff only (measurement run)", "value": None, "unit": "GB/s",
                    "config": {"workload": WORKLOADS["c3"]["desc"], "blobs_this_rank": n,
                               "emulated_world": shard_world, "emulated_rank": shard_rank,
                               "longest_blob": int(max(lens))}})
        res["tail_handoff"] = run_tail_handoff(a, D, T, ids, lens, P, int(sum(c3_lengths(a.blobs or 20000))),
                                               None, None)
        return
    wr = WindowedRun(D, ids, lens, P, a.window_gib << 30,
                     cap=n if a.no_admission else (a.live_cap or None))
    T.barrier()
    with D.KernelTimer():
        t0 = time.perf_counter()
        wr.run()
        T.barrier()
        t1 = time.perf_counter()
        sha_n, sha_ms = D.KernelTimer.stats("sha256_multi")
        crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
        gen_n, gen_ms = D.KernelTimer.stats("synth_fill")
    elapsed = T.timed_region(t1 - t0)
    bytes_rank = int(sum(lens))
    total_bytes = int(sum(c3_lengths(a.blobs or 20000)))
    cb = wr.cb
    res.update({"metric": "metainfo+digest GB/s (C3, device-generated windows)",
                "value": round(total_bytes / elapsed / 1e9, 3), "unit": "GB/s", "steps": 1,
                "ms_per_step": round(elapsed * 1e3, 3), "higher_is_better": True, "scaling": "strong",
                "dtype": "u8", "data": "synthetic (generated on the device per window, inside the timed region)",
                "config": {"workload": WORKLOADS["c3"]["desc"], "blobs_total": a.blobs or 20000,
                           "blobs_this_rank": n, "bytes_this_rank": bytes_rank, "bytes_total": total_bytes,
                           "windows": len(wr.wins), "window_bytes": wr.W, "live_cap": int(wr.cap), "piece_length": P,
                           "longest_blob": max(lens), "parallelism": f"LPT blob shard x{shard_world}, no collective",
                           **({"emulated_world": shard_world,
                               "emulated_rank": shard_rank,
                               "emulation": f"rank {shard_rank}'s shard of a {shard_world}-GPU run on one GPU; value = "
                                            f"all {shard_world} shards' bytes / this shard's time"
                                            + (" (it holds the longest blob)" if shard_rank == 0 else "")}
                             if a.emulate_world else {})},
                "kernels": {"sha256_multi": {"launches": sha_n, "total_ms": round(sha_ms, 1)},
                            "crc32_pieces": {"launches": crc_n, "total_ms": round(crc_ms, 1)},
                            "synth_fill": {"launches": gen_n, "total_ms": round(gen_ms, 1)}},
                "note": "bounded below by the longest blob's sequential SHA-256 chain (longest_blob / per-stream "
                        "rate) at any GPU count"})
    # Dominant kernel by device time: SHA-256 over every window (bytes / summed launch time).
    if sha_n:
        gbps = bytes_rank / (sha_ms / 1e3) / 1e9
        roof = roofline_obj("sha256_multi", gbps, sha_ms / sha_n, bytes_rank / sha_n, None)
        roof["chain"] = {"peak": None, "frac": None}
        # The chain bound: no schedule finishes before the longest blob's chain, which runs
        # at the per-stream ISA ceiling of the plan the first (largest) window takes.
        lanes = D.sha_lanes_per_stream(int(min(wr.cap, n)))
        if lanes in (2, 8) and not a.no_ceiling:
            import ctypes as C
            import sha_isa
            try:
                isa = sha_isa.count(D.lib._name, lanes)
                mhz = C.c_double()
                D.check(D.lib.krk_device_clock_mhz(None, C.byref(mhz)))
                ceil = sha_isa.ceiling_mbps(isa, mhz.value)
                peak = bytes_rank / (max(lens) / (ceil * 1e6)) / 1e9
                roof["chain"] = {"peak": round(peak, 2), "frac": round(gbps / peak, 4)}
                roof.update({"chain_bound": {"longest_blob": max(lens), "lanes_per_stream": lanes,
                                             "ceiling_per_stream_MBps": round(ceil, 2),
                                             "clock_mhz": round(mhz.value, 1),
                                             "source": "tools/sha_isa.py VALU per block x 4 cycles, idle clock"}})
            except Exception as e:  # tools missing on the box: report, never guess
                roof["ceiling_error"] = f"{type(e).__name__}: {e}"
        roof["note"] = ("peak/frac: the HBM roofline (8 TB/s spec); achieved = SHA bytes / summed SHA launch time. "
                        "What bounds it is VALU issue along the longest chain (DESIGN.md 4.2): chain.peak = the bytes "
                        "over the longest blob's chain at the per-stream ISA ceiling (no schedule beats it); the "
                        "windows shrink as blobs finish, so late launches carry few streams")
        res["roofline"] = roof
    dg = cb.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
    sums = cb.sums.to_host(np.uint32, max(cb.total_pieces, 1))
    if rank == 0 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_c3(ids, lens, P, dg, sums, cb.sums_off)
    if rank == 0:  # spot-check three blobs against the one-shot device path
        pick = sorted({0, n // 2, n - 1})
        wr.close()
        arena = D.BlobArena([lens[i] for i in pick], P, blob_ids=[ids[i] for i in pick])
        out = D.BatchOutputs(arena)
        D.metainfo_digest(arena, out)
        D.synchronize()
        ref = out.digests.to_host(np.uint8, 32 * len(pick)).reshape(-1, 32)
        rs = out.sums.to_host(np.uint32, arena.total_pieces)
        ok = all(bytes(dg[i]) == bytes(ref[k]) for k, i in enumerate(pick))
        for k, i in enumerate(pick):
            o, ro, cnt = int(cb.sums_off[i]), int(arena.sums_off[k]), int(arena.n_pieces[k])
            ok = ok and np.array_equal(sums[o:o + cnt], rs[ro:ro + cnt])
        res["spot_check_matches_one_shot"] = bool(ok)
    wr.close()
    # the host lane before the tail handoff: the lane loses 15-35 % when it runs second in a
    # process (cause not isolated, profiles/r06/c3_w8_leg_order.jsonl); the handoff lost its
    # 7-20 % second only to the copy engines' half-rate window after the lane freed its
    # memory, which settle_dma now waits out
    if a.host_lane:
        res["host_offload"] = run_host_lane(a, D, T, ids, lens, P, total_bytes, dg, sums)
    if a.tail_handoff:
        res["tail_handoff"] = run_tail_handoff(a, D, T, ids, lens, P, total_bytes, dg, sums)
    if not a.no_e2e:
        res["end_to_end"] = c3_end_to_end(D, T, world, rank)


_SETTLE = {}


def settle_dma(D, max_s=15.0):
    """Wait until device-to-host copies run at the calibrated rate again before a leg starts.
    After a leg frees tens of GB of device memory, D2H copies run at half rate (30.3 against
    56.5 GB/s) for ~4 s and then jump back (profiles/r06/d2h_after_lane_timeline.json) -- the
    copy engines busy with something of the driver's after the free; a leg that started
    inside that window lost 7-20 % (c3_w8_leg_order.jsonl).  Returns the seconds waited."""
    import ctypes as C
    if not _SETTLE:
        _SETTLE["src"] = D.DeviceBuffer(64 << 20)
        _SETTLE["dst"] = [D.PinnedArray((64 << 20,), np.uint8) for _ in range(4)]
        s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(s)))
        _SETTLE["s"] = s
    want = 0.85 * D.planner_rates()["d2h_bps"]
    t0 = time.perf_counter()
    while True:
        t1 = time.perf_counter()
        for b in _SETTLE["dst"]:
            D.check(D.lib.krk_memcpy_d2h_async(C.c_void_p(b.ptr), C.c_void_p(_SETTLE["src"].ptr), 64 << 20,
                                               _SETTLE["s"]))
        D.check(D.lib.krk_stream_sync(_SETTLE["s"]))
        r = 4 * (64 << 20) / (time.perf_counter() - t1)
        if r >= want or time.perf_counter() - t0 > max_s:
            return round(time.perf_counter() - t0, 3)
        time.sleep(0.1)


def run_host_lane(a, D, T, ids, lens, P, total_bytes, dg, sums):
    """C3 with the host lane (kraken_amd.windowed): the K longest blobs of the shard are
    generated into a device buffer of their own, their piece CRCs run on the GPU and their
    SHA-256 on host threads reading HBM, while the windows run the rest.  GPU + host
    throughput: reported beside the GPU-only value, never as it.  K from the planner
    (windowed.host_lane_plan over krk_planner_rates) unless --host-lane-k."""
    from kraken_amd.windowed import WindowedRun, host_lane_plan, window_stream_cap
    threads = max(1, host_cores() - 1)  # one core stays with the window loop
    W = a.window_gib << 30
    cap = len(lens) if a.no_admission else (a.live_cap or window_stream_cap(D, len(lens)))
    rates = D.planner_rates()
    k, model_s, model0_s = host_lane_plan(D, lens, W, cap, threads, rates=rates)
    if a.host_lane_k >= 0:
        k = min(a.host_lane_k, len(lens))
    out = {"blobs_on_host": int(k), "threads": threads,
           "modelled_s": round(model_s, 3), "modelled_gpu_only_s": round(model0_s, 3),
           "planner_rates": {"sha_stream_MBps": [round(x / 1e6, 2) for x in rates["sha_stream_bps"]],
                             "host_sha_GBps_per_thread": round(rates["host_sha_bps"] / 1e9, 3),
                             "d2h_GBps": round(rates["d2h_bps"] / 1e9, 2), "source": rates["source"]},
           "what": "GPU + host: the longest blobs hashed by host threads reading them out of HBM (SHA-NI) while "
                   "the GPU windows run the rest; their piece CRCs stay on the GPU"}
    if k == 0:
        out["note"] = "the planner keeps every blob on the GPU (the lane would not shorten the run by 2 %)"
        return out
    wr = WindowedRun(D, ids, lens, P, W, cap=cap if (a.no_admission or a.live_cap) else None,
                     host_lane=(k, threads), device=a.device)
    out["settle_s"] = settle_dma(D)
    T.barrier()
    t0 = time.perf_counter()
    wr.run()
    T.barrier()
    el = T.max_over_ranks(time.perf_counter() - t0)
    n = len(lens)
    dg2 = wr.cb.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
    s2 = wr.cb.sums.to_host(np.uint32, max(wr.cb.total_pieces, 1))
    wr.close()
    out.update({"value": round(total_bytes / el / 1e9, 3), "unit": "GB/s", "ms_per_step": round(el * 1e3, 3),
                "host_bytes": int(sum(lens[i] for i in wr.lane_blobs)), "lane_s": round(wr.lane_seconds, 3),
                "windows": len(wr.wins),
                "matches_gpu_only": bool(np.array_equal(dg2, dg) and np.array_equal(s2, sums))})
    return out


def run_tail_handoff(a, D, T, ids, lens, P, total_bytes, dg, sums):
    """C3 with the tail handoff (kraken_amd.windowed.TailHandoffRun): every chain starts in
    the windows (the threads start on the longest ones whole) and host threads steal the
    chains with the most bytes left at window boundaries, from the midstates in HBM; the
    stolen chains' remaining piece CRCs stay on the GPU.  GPU + host throughput, reported
    beside the GPU-only value (never as it), with the same policy modelled on the planner's
    rates (windowed.simulate_tail_handoff) and the outputs compared with the GPU-only run's."""
    from kraken_amd.windowed import TAIL_CHUNK, TailHandoffRun, simulate_tail_handoff, window_stream_cap
    threads = a.tail_threads or max(1, host_cores() - 1)  # one core stays with the window loop
    cap = len(lens) if a.no_admission else (a.live_cap or window_stream_cap(D, len(lens)))
    live = min(cap, len(lens))
    # windows of <= 4 MiB a live chain (a ~70 ms SHA launch at eight lanes): a chain is handed
    # over at a window boundary, so short windows keep the threads from waiting on one
    W = int(min(a.window_gib << 30, live * TAIL_CHUNK))
    rates = D.planner_rates()
    model = simulate_tail_handoff(lens, W, cap, threads, rates, max_chunk=TAIL_CHUNK)
    gpu_model = simulate_tail_handoff(lens, W, cap, 0, rates, max_chunk=TAIL_CHUNK)
    out = {"threads": threads, "window_bytes": W, "live_cap": int(cap),
           "model": {"end_s": round(model["end_s"], 3), "gpu_windows_end_s": round(model["gpu_end_s"], 3),
                     "host_bytes": int(model["host_bytes"]), "takeovers": int(model["takeovers"]),
                     "value_GBps": round(total_bytes / model["end_s"] / 1e9, 3),
                     "thread_rate_GBps": round(model["thread_rate_Bps"] / 1e9, 3),
                     "gpu_only_end_s": round(gpu_model["end_s"], 3),
                     "modelled_gain": round(gpu_model["end_s"] / model["end_s"], 3)},
           # the handoff's measured end runs 1.03-1.08x its model at 8 and 4 GPUs, more as the
           # windows turn throughput-bound (profiles/r06): below a modelled gain of ~1.2 the
           # windows' serialised CRCs and the threads' midstate waits eat most of the gain (C3 at
           # N=1: modelled 1.08, measured 0.91x the GPU alone; 2 GPUs: modelled 1.15, 1.03-1.07x)
           "planner_uses_it": bool(gpu_model["end_s"] / model["end_s"] >= 1.2),
           "planner_rates": {"sha_stream_MBps": [round(x / 1e6, 2) for x in rates["sha_stream_bps"]],
                             "host_sha_GBps_per_thread": round(rates["host_sha_bps"] / 1e9, 3),
                             "d2h_GBps": round(rates["d2h_bps"] / 1e9, 2), "source": rates["source"]},
           "what": "GPU + host: host threads (SHA-NI) steal the chains with the most bytes left at window "
                   "boundaries from the windows' midstates in HBM; piece CRCs all on the GPU"}
    from kraken_amd.windowed import TAIL_PIECE, TAIL_RING
    tr = TailHandoffRun(D, ids, lens, P, W, threads, cap=cap if (a.no_admission or a.live_cap) else None,
                        device=a.device, piece=(a.tail_piece_mib << 20) if a.tail_piece_mib else TAIL_PIECE,
                        ring=a.tail_ring or TAIL_RING, crc_after_sha=False if a.tail_crc_beside_sha else None)
    out["settle_s"] = settle_dma(D)
    T.barrier()
    t0 = time.perf_counter()
    tr.run()
    T.barrier()
    el = T.max_over_ranks(time.perf_counter() - t0)
    n = len(lens)
    dg2 = tr.cb.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
    s2 = tr.cb.sums.to_host(np.uint32, max(tr.cb.total_pieces, 1))
    tr.close()
    out.update({"value": round(total_bytes / el / 1e9, 3), "unit": "GB/s", "ms_per_step": round(el * 1e3, 3),
                "measured_over_model": round(el / model["end_s"], 4), **tr.stats,
                **({"matches_gpu_only": bool(np.array_equal(dg2, dg) and np.array_equal(s2, sums))}
                   if dg is not None else {})})
    return out


def run_hrw(a, D, T, rank, world, res):
    n = a.blobs or 1_000_000
    N, R = a.nodes, 3
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(N)]
    healthy = np.ones(N, dtype=np.uint8)
    rng = np.random.default_rng(0xC5 + rank)
    dig = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(dig.reshape(-1))
    # Owner lists as uint8 node indices (krk_ring_locations_u8_dev) when the ring has
    # <= 255 nodes: a quarter of the bytes to write and to copy back; int32 otherwise.
    compact = N <= 255 and not a.hrw_int32
    isz = 1 if compact else 4
    locs = D.DeviceBuffer(n * R * isz)
    counts = D.DeviceBuffer(n)
    pin = D.PinnedArray((n, R), np.uint8 if compact else np.int32)  # owner lists gathered to pinned host memory
    locs_h = pin.a
    place = D.ring_locations_u8_dev if compact else D.ring_locations_dev
    # A step = the placement call, the owner lists' copy into pinned host memory queued
    # behind it on the same stream, and one wait for that stream (how a caller uses it: the
    # lists are on the host when the step ends).  Serial: each step's lists on the host
    # before the next is enqueued.  `back_to_back` then enqueues step k + 1 on the other
    # stream (its own outputs) before waiting for step k, so the host's enqueue and each
    # copy overlap the neighbour's kernel (a placement service draining a queue of batches).
    import ctypes as C
    streams = [C.c_void_p(), C.c_void_p()]
    for st in streams:
        D.check(D.lib.krk_stream_create(C.byref(st)))
    outs = [(locs, counts, pin), (D.DeviceBuffer(n * R * isz), D.DeviceBuffer(n),
                                  D.PinnedArray((n, R), np.uint8 if compact else np.int32))]

    enq_s = [0.0]

    def enqueue(k):
        lo, co, pi = outs[k & 1]
        t = time.perf_counter()
        place(dbuf, n, labels, healthy, R, lo, co, stream=streams[k & 1])
        pi.fill_from_async(lo, streams[k & 1])
        enq_s[0] += time.perf_counter() - t

    def run(nsteps, serial, enq=enqueue):
        for k in range(nsteps):
            enq(k)
            if serial:
                D.check(D.lib.krk_stream_sync(streams[k & 1]))
            elif k:
                D.check(D.lib.krk_stream_sync(streams[(k - 1) & 1]))
        if nsteps:
            D.check(D.lib.krk_stream_sync(streams[(nsteps - 1) & 1]))

    run(a.warmup, True)
    T.barrier()
    enq_s[0] = 0.0
    with D.KernelTimer():
        t0 = time.perf_counter()
        run(a.steps, True)
        T.barrier()
        t1 = time.perf_counter()
        hn, hms = D.KernelTimer.stats("hrw_order")
        gn, gms = D.KernelTimer.stats("hrw_gather")
    elapsed = T.timed_region(t1 - t0)
    enqueue_us = enq_s[0] / max(a.steps, 1) * 1e6
    locs_h = outs[(a.steps - 1) & 1][2].a if a.steps else locs_h
    want_locs = locs_h.copy()
    T.barrier()
    t2 = time.perf_counter()
    run(a.steps, False)
    T.barrier()
    el_b2b = T.max_over_ranks(time.perf_counter() - t2)
    b2b_ok = all(np.array_equal(outs[i][2].a, want_locs) for i in range(min(2, a.steps)))
    try:
        # The same steps with locs in page-locked host memory: the gather writes the owner lists
        # over PCIe as it goes and the step has no copy-back (counts stay in HBM, as in the copy
        # path: the 0xFF padding already tells a list's length).
        mouts = [(D.PinnedArray((n, R), np.uint8 if compact else np.int32), D.DeviceBuffer(n)) for _ in range(2)]

        def enqueue_mapped(k):
            lo, co = mouts[k & 1]
            place(dbuf, n, labels, healthy, R, lo, co, stream=streams[k & 1])

        run(a.warmup, True, enqueue_mapped)
        T.barrier()
        with D.KernelTimer():
            t3 = time.perf_counter()
            run(a.steps, True, enqueue_mapped)
            T.barrier()
            t4 = time.perf_counter()
            mg_n, mg_ms = D.KernelTimer.stats("hrw_gather")
        el_m = T.max_over_ranks(t4 - t3)
        m_ok = bool(np.array_equal(mouts[(a.steps - 1) & 1][0].a, want_locs)) if a.steps else True
        T.barrier()
        t5 = time.perf_counter()
        run(a.steps, False, enqueue_mapped)
        T.barrier()
        el_mb = T.max_over_ranks(time.perf_counter() - t5)
        m_ok = m_ok and all(np.array_equal(mouts[i][0].a, want_locs) for i in range(min(2, a.steps)))
        mg_avg = mg_ms / max(mg_n, 1)
        out_bytes = n * isz * R
        mapped = {"value": round(world * n * a.steps / el_m, 1), "unit": "digests/s",
                  "ms_per_step": round(el_m / a.steps * 1e3, 3),
                  "back_to_back": {"value": round(world * n * a.steps / el_mb, 1),
                                   "ms_per_step": round(el_mb / a.steps * 1e3, 3)},
                  "hrw_gather": {"launches": mg_n, "avg_ms": round(mg_avg, 4),
                                 "host_write_GBps": round(out_bytes / (mg_avg / 1e3) / 1e9, 2) if mg_avg else None},
                  "locs_match_copy_path": m_ok,
                  "what": "locs in krk_host_alloc memory: the gather writes the owner lists over PCIe (no "
                          "copy-back; counts in HBM as in the copy path); host_write_GBps = owner-list bytes / "
                          "gather time"}
    except Exception as e:  # reported, never hidden: the line keeps the copy path's numbers
        mapped = {"error": f"{type(e).__name__}: {e}"}
    copy_back = {"value": round(world * n * a.steps / elapsed, 1), "unit": "digests/s",
                 "ms_per_step": round(elapsed / a.steps * 1e3, 3), "host_enqueue_us": round(enqueue_us, 1),
                 "hrw_gather": {"launches": gn, "avg_ms": round(gms / max(gn, 1), 4)},
                 "back_to_back": {"value": round(world * n * a.steps / el_b2b, 1),
                                  "ms_per_step": round(el_b2b / a.steps * 1e3, 3), "locs_match_serial": b2b_ok},
                 "what": "locs and counts in HBM, the owner lists copied into pinned host memory on the same "
                         "stream behind the gather (hipMemcpyAsync D2H), one wait a step; back_to_back: step k+1 "
                         "enqueued on the other stream (its own outputs) before the host waits for step k"}
    # The step `value` times: the library path that leaves the owner lists on the host --
    # written there by the gather when that is measured faster (and it works), else copied.
    use_mapped = "error" not in mapped and mapped["value"] >= copy_back["value"]
    main = mapped if use_mapped else copy_back
    res.update({"metric": "hashring placement digests/s (C5)", "value": main["value"],
                "unit": "digests/s", "steps": a.steps, "ms_per_step": main["ms_per_step"],
                "higher_is_better": True, "scaling": "weak", "dtype": "u64+f64",
                "data": "synthetic (seeded random 32-byte digests)",
                "config": {"workload": WORKLOADS["c5"]["desc"], "digests_per_gpu": n, "nodes": N,
                           "max_replica": R, "mode": "device-resident digests (65,536-shard table + gather), owner "
                                                     "lists on the host at the end of each step: "
                                                     + ("written by the gather into page-locked host memory"
                                                        if use_mapped else "copied back into pinned host memory"),
                           "owner_index_bytes": isz},
                "kernels": {"hrw_order": {"launches": hn, "avg_ms": round(hms / max(hn, 1), 3)},
                            "hrw_gather": main["hrw_gather"]},
                "back_to_back": main["back_to_back"], "mapped_outputs": mapped, "copy_back": copy_back})
    # Roofline of the per-digest kernel.  Device outputs: HBM-bound (32-B digest record in, R
    # owner indices + a count out).  Outputs in host memory: the gather's stores cross the
    # link, so the link's D2H rate bounds it.  The shard-table kernel's work is fixed (65,536
    # ShardIDs x N scores: murmur3 + Go math.Log, VALU/f64-bound, not per-digest).
    g_avg = gms / max(gn, 1)
    per_digest = 32 + isz * R + 1
    roof_dev = roofline_obj("hrw_gather", n * per_digest / (g_avg / 1e3) / 1e9 if g_avg else 0.0, g_avg,
                            n * per_digest, load_traffic(a.pmc_json, "c5", n).get("hrw_gather") if compact else None)
    roof_dev["note"] = (f"device outputs (the copy_back leg); algorithmic bytes per digest = {per_digest} (32-B "
                        f"digest record + {R} x {isz}-B owner indices + 1-B count); the hrw_order kernel (65,536-shard "
                        f"table, {round(hms / max(hn, 1), 3)} ms) is VALU-bound and independent of the digest count")
    if use_mapped:
        d2h = D.planner_rates()["d2h_bps"] / 1e9
        ach = mapped["hrw_gather"]["host_write_GBps"] or 0.0
        res["roofline"] = {"kernel": "hrw_gather", "bound": "host link (PCIe writes)", "achieved": ach,
                           "peak": round(d2h, 3), "unit": "GB/s", "frac": round(ach / d2h, 4) if d2h else None,
                           "traffic": None, "avg_launch_ms": mapped["hrw_gather"]["avg_ms"],
                           "algorithmic_bytes_per_launch": n * isz * R,
                           "peak_source": "pinned D2H measured on this device (krk_planner_rates_get: d2h_bps)",
                           "note": "the gather writes the owner lists (R x 1 B a digest) into page-locked host memory "
                                   "over PCIe: achieved = those bytes / average gather time; its HBM side (32-B digest "
                                   "records) is roofline_device_outputs"}
        res["roofline_device_outputs"] = roof_dev
    else:
        res["roofline"] = roof_dev
    if rank == 0 and not a.no_cpu_baseline:
        cbl, cl, cc = cpu_baseline_hrw(dig, labels, healthy, R, a.cpu_seconds)
        got = locs_h[:cl.shape[0]].astype(np.int32)
        if compact:
            got[got == 255] = -1
        cbl["outputs_match_gpu"] = bool(np.array_equal(cl, got))
        res["cpu_baseline"] = cbl
    if rank == 0 and world == 1 and not a.no_sweep:
        res["sweep"] = hrw_sweep(D, dbuf, dig, n, a.steps)


def hrw_sweep(D, dbuf, dig, n, steps):
    """SURVEY.md 8(d) C5 grid: N in {3, 5, 16, 64} origins x MaxReplica in {2, 3} x
    healthy = all / a seeded 75 % subset, plus the weighted variant (100/200/400/800).
    Each point: digests/s over `steps` timed calls, and its first 2,048 digests
    checked against the oracle's GetOrderedNodes + Locations filter."""
    from oracle import oracle as O  # the checker (test infrastructure)
    O.build()
    points = [(N, R, hf, False) for N in (3, 5, 16, 64) for R in (2, 3) for hf in (1.0, 0.75)]
    points += [(16, 3, 1.0, True), (64, 3, 0.75, True)]
    out = []
    for N, R, hf, weighted in points:
        labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(N)]
        weights = [[100, 200, 400, 800][i % 4] if weighted else 100 for i in range(N)]
        healthy = np.ones(N, dtype=np.uint8)
        if hf < 1.0:
            rng = np.random.default_rng(0x75 + N)
            healthy[rng.choice(N, N - int(round(N * hf)), replace=False)] = 0
        locs = D.DeviceBuffer(n * R)
        counts = D.DeviceBuffer(n)
        pin = D.PinnedArray((n, R), np.uint8)  # compact owner lists (every grid ring has <= 64 nodes)
        D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, locs, counts, weights=weights)
        D.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):  # same step as the headline C5 line: results gathered to host
            D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, locs, counts, weights=weights)
            D.synchronize()
            pin.fill_from(locs)
        el = time.perf_counter() - t0
        got = pin.a
        cnt = counts.to_host(np.uint8, n)
        ok, memo = True, {}
        for i in range(2048):
            key = bytes(dig[i, :2]).hex()
            if key not in memo:
                order = O.hrw_ordered(key, labels, weights)
                memo[key] = O.ring_locations(order, healthy, R)
            want = list(memo[key])
            ok = ok and int(cnt[i]) == len(want) and got[i, :len(want)].tolist() == want
        out.append({"nodes": N, "max_replica": R, "healthy": int(healthy.sum()), "weighted": weighted,
                    "digests_per_s": round(n * steps / el, 1), "oracle_match_first_2048": bool(ok)})
    return out


def run_files(a, D, T, rank, world, res):
    """The f3 file leg (krk_metainfo_digest_files): the C3 length law / 64 from
    files on the box's disk (page cache warm after the first pass).  value = blob bytes / time
    of one call, every byte read once and over PCIe once (GPU only: the host offload off);
    beside it the same batch from pinned host memory (krk_metainfo_digest_host) and the
    library's default (AUTO offload).  Digests and piece sums of the three runs are equal and
    sampled blobs equal the oracle."""
    import resource
    import shutil
    import tempfile
    n, SRC, P = a.blobs or 16384, 64, 4 << 20
    lens = c3_lengths(n, scale=64)
    top = max(lens)
    d = tempfile.mkdtemp(prefix=f"krk_files_r{rank}_")
    try:
        srcs = []
        for k in range(SRC):  # device-generated content, copied down and written once
            buf = D.DeviceBuffer(top)
            D.check(D.lib.krk_synth_fill_dev(buf.ptr, (3 << 40) + rank * SRC + k, 0, top, 0, None))
            D.synchronize()
            x = buf.to_host(np.uint8, top)
            buf.free()
            with open(os.path.join(d, f"src{k}"), "wb") as f:
                f.write(memoryview(x))
            srcs.append(x)
        paths = [os.path.join(d, f"src{i % SRC}") for i in range(n)]
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        resource.setrlimit(resource.RLIMIT_NOFILE, (min(hard, 1 << 20), hard))  # as Go's runtime does
        total = int(sum(lens))
        for _ in range(a.warmup):
            D.metainfo_digest_files(paths, lens, P)
        T.barrier()
        with D.KernelTimer():
            c_f = cpu_seconds()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                sums_f, dg_f = D.metainfo_digest_files(paths, lens, P)
            T.barrier()
            t1 = time.perf_counter()
            c_f = cpu_seconds() - c_f
            st = D.windows_last_call()
            sha_n, sha_ms = D.KernelTimer.stats("sha256_multi")
            crc_n, crc_ms = D.KernelTimer.stats("crc32_pieces")
        elapsed = T.timed_region(t1 - t0)
        value = world * total * a.steps / elapsed / 1e9
        # the same bytes from pinned host memory, and the library's default (AUTO offload)
        pins = []
        for x in srcs:
            pa = D.PinnedArray((x.size,), np.uint8)
            pa.a[:] = x
            pins.append(pa)
        datas = [pins[i % SRC].a[:lens[i]] for i in range(n)]
        D.metainfo_digest_host(datas, P)
        # pinned blobs: the library's default gathers the wide windows from the caller's pages
        # (one launch a window); KRK_HOST_GATHER=0's staging copy beside it
        pinned_paths = {}
        for name, mode in (("staged", 0), ("gather", -1)):
            D.set_host_gather(mode)
            try:
                T.barrier()
                c0, t0 = cpu_seconds(), time.perf_counter()
                sums_p, dg_p = D.metainfo_digest_host(datas, P)
                cpu_p = cpu_seconds() - c0
                T.barrier()
                el_p = T.max_over_ranks(time.perf_counter() - t0)
                st_p = D.windows_last_call()
            finally:
                D.set_host_gather(-1)
            pinned_paths[name] = {"GBps": round(world * total / el_p / 1e9, 3),
                                  "host_cpu_s_per_GB": round(cpu_p / (total / 1e9), 4),
                                  "windows": st_p["windows"], "gather_windows": st_p["gather_windows"]}
        D.set_sha_host_offload(-1)
        try:
            T.barrier()
            t0 = time.perf_counter()
            sums_a, dg_a = D.metainfo_digest_files(paths, lens, P)
            T.barrier()
            el_a = T.max_over_ranks(time.perf_counter() - t0)
            st_a = D.windows_last_call()
        finally:
            D.set_sha_host_offload(0)
        same = (np.array_equal(dg_f, dg_p) and np.array_equal(dg_f, dg_a) and
                all(np.array_equal(x, y) and np.array_equal(x, z) for x, y, z in zip(sums_f, sums_p, sums_a)))
        from oracle import oracle as O  # checker only
        O.build()
        import hashlib
        L = np.asarray(lens)
        ok = True
        for i in sorted({int(L.argmin()), int(L.argmax()), n // 2}):
            x = srcs[i % SRC][:lens[i]]
            ok = ok and bytes(dg_f[i]) == hashlib.sha256(x.tobytes()).digest() and np.array_equal(
                sums_f[i], O.calc_piece_sums(x, P)[1])
        del pins, datas
        cb = None
        if rank == 0 and not a.no_cpu_baseline:
            # the reference's two reads of every file on the CPU budget: uploader.verify's
            # Digester over the upload file, then Generate's calcPieceSums over the cache file
            t_c, s_c, off_c, dg_c = O.baseline_files(paths, lens, P, node_cores(), passes=3)
            same_c = bool(np.array_equal(dg_c, dg_f)) and all(
                np.array_equal(s_c[int(off_c[i]):int(off_c[i + 1])], sums_f[i]) for i in range(n))
            cb = {"value": round(total / t_c / 1e9, 3), "unit": "GB/s", "cores": node_cores(),
                  "cores_source": CORES_SOURCE, "kind": "port",
                  "seconds": round(t_c, 3), "outputs_match_gpu": same_c,
                  "sample": f"all {n} files of the pass (page cache warm): Digester.FromReader then calcPieceSums "
                            "over each file, 32 KiB reads, SHA-NI and PCLMUL, one file per thread "
                            "(oracle/oracle.c orc_baseline_files)"}
    finally:
        shutil.rmtree(d, ignore_errors=True)
    if a.cold_gib > 0:
        res["cold"] = files_cold_leg(a, D, T, rank, world, P)
    res.update({"metric": "upload verify + metainfo from files, GB/s (end-to-end, host link)",
                "value": round(value, 3), "unit": "GB/s", "steps": a.steps,
                "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
                "dtype": "u8", "data": "synthetic (device-generated splitmix64 sources written to local files)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "blobs_per_gpu": n, "bytes_per_gpu": total,
                           "piece_length": P, "mode": "files -> pinned windows -> GPU (offload off)",
                           "parallelism": f"blob-sharded x{world}, no collective"},
                "roofline": link_roofline(D, value, "files", n, world=world),
                "windows": st, "kernels": {"sha256_multi": {"launches": sha_n, "avg_ms": round(sha_ms / max(sha_n, 1), 3)},
                                           "crc32_pieces": {"launches": crc_n, "avg_ms": round(crc_ms / max(crc_n, 1), 3)}},
                "host_cpu_s_per_GB": round(c_f / a.steps / (total / 1e9), 4),
                "pinned_host_memory": {"value": round(world * total / el_p / 1e9, 3), "unit": "GB/s",
                                       "roofline": link_roofline(D, world * total / el_p / 1e9, world=world),
                                       "windows": st_p, "paths": pinned_paths,
                                       "what": "the same blobs from pinned host memory (krk_metainfo_digest_host): "
                                               "value = the library's default (wide windows gathered from the "
                                               "caller's pages, gather.hip); paths.staged = KRK_HOST_GATHER=0 "
                                               "(pinned -> pinned window copies, then the DMA)"},
                "default_offload": {"value": round(world * total / el_a / 1e9, 3), "unit": "GB/s",
                                    "host_blobs": st_a["host_blobs"],
                                    "what": "krk_metainfo_digest_files with the library's default host offload (AUTO)"},
                "outputs_equal_across_paths": bool(same), "oracle_sampled_match": bool(ok)})
    if cb:
        res["cpu_baseline"] = cb


# The library's DEFAULTS in a fresh process (no knob, no KRK_ environment): a C1-shaped
# batch through krk_metainfo_digest_dev and one 1 GiB NewMetaInfo piece stream of 4 MiB
# reads, against one host thread's SHA-NI / PCLMUL time of the same bytes.  The outputs and
# placements are asserted here (tests/test_gpu_defaults.py runs it as a parity test); the
# times are the `--workload defaults` line's.
DEFAULTS_PROBE = r"""
import ctypes as C, hashlib, json, sys, time, zlib
import numpy as np
sys.path.insert(0, ".")
from kraken_amd import device as D
from kraken_amd._capi import KRK_OFFLOAD_AUTO, KRK_PLACE_HOST, check, lib
RUNS = int(sys.argv[1])
D.set_device(0)
t = C.c_int(0)
check(lib.krk_sha_host_offload(C.byref(t)))
assert t.value == KRK_OFFLOAD_AUTO, t.value
L, P = 1 << 30, 4 << 20
arena = D.BlobArena([L], P, blob_ids=[7])
out = D.BatchOutputs(arena)
host = arena.buf.to_host(np.uint8, L)
res = {"blob_bytes": L, "piece_length": P, "runs": RUNS}

def best(f, k=RUNS):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    return min(ts)
# one host thread, the same bytes: SHA-NI (krk_host_sha256) and PCLMUL (krk_host_crc32_update)
o32 = (C.c_uint8 * 32)()
res["host_sha_1thread_s"] = best(lambda: lib.krk_host_sha256(host.ctypes.data, L, o32))
want_dg = hashlib.sha256(host).digest()
assert bytes(o32) == want_dg
c = C.c_uint32()
res["host_crc_1thread_s"] = best(lambda: lib.krk_host_crc32_update(0, host.ctypes.data, L, C.byref(c)))
assert c.value == zlib.crc32(host)

def c1():  # C1 through the device-resident drop-in, defaults
    D.metainfo_digest(arena, out)
    D.synchronize()
res["c1_metainfo_digest_dev_s"] = best(c1)
dg = out.digests.to_host(np.uint8, 32)
sums = out.sums.to_host(np.uint32, arena.total_pieces)
want_sums = [zlib.crc32(host[i:i + P]) for i in range(0, L, P)]
assert bytes(dg) == want_dg
assert sums.tolist() == want_sums
res["digest_ok"] = res["sums_ok"] = True

placement = []
def stream():  # one NewMetaInfo stream, 4 MiB reads, defaults
    s = C.c_void_p()
    check(lib.krk_piece_stream_begin(P, C.byref(s)))
    w = C.c_int(-1)
    check(lib.krk_piece_stream_placement(s, C.byref(w)))
    placement.append(w.value)
    base = host.ctypes.data
    for a in range(0, L, 4 << 20):
        check(lib.krk_piece_stream_update(s, base + a, min(4 << 20, L - a)))
    ns, ln = C.c_uint64(), C.c_uint64()
    got = (C.c_uint32 * 256)()
    check(lib.krk_piece_stream_end(s, got, 256, C.byref(ns), C.byref(ln)))
    lib.krk_piece_stream_free(s)
    assert ns.value == 256 and ln.value == L
    stream.sums = list(got)
res["stream_s"] = best(stream)
assert stream.sums == want_sums
assert all(p == KRK_PLACE_HOST for p in placement), placement
res["stream_placement"] = "host"
res["stream_GBps"] = L / res["stream_s"] / 1e9
res["host_crc_1thread_GBps"] = L / res["host_crc_1thread_s"] / 1e9
res["host_sha_1thread_GBps"] = L / res["host_sha_1thread_s"] / 1e9
res["c1_GBps"] = L / res["c1_metainfo_digest_dev_s"] / 1e9
res["c1_ratio_to_host_sha"] = res["c1_metainfo_digest_dev_s"] / res["host_sha_1thread_s"]
print(json.dumps(res))
"""


def run_defaults_probe(runs=3):
    """DEFAULTS_PROBE in a fresh child process with every KRK_ variable removed."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("KRK_")}
    r = subprocess.run([sys.executable, "-c", DEFAULTS_PROBE, str(runs)], capture_output=True, text=True, cwd=ROOT,
                       env=env, timeout=600)
    if r.returncode != 0:
        raise RuntimeError("defaults probe failed: " + r.stdout[-2000:] + r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def run_defaults(a, D, T, rank, world, res):
    """The library's defaults on the two single-stream drop-ins (C1's NewMetaInfo + digest,
    one NewMetaInfo piece stream), each the best of `steps` runs in a fresh process, against
    one host thread of the reference's own placement on the same bytes.  value = C1 GB/s
    with the defaults; the line carries the VERDICT r03 item 1 criteria as measured booleans
    (C1 within 1.2x of one SHA-NI thread, the stream at least one PCLMUL thread)."""
    p = run_defaults_probe(runs=max(1, a.steps))
    el = T.timed_region(p["c1_metainfo_digest_dev_s"])
    res.update({"metric": "defaults: C1 NewMetaInfo+digest GB/s (library defaults, fresh process)",
                "value": round(world * p["blob_bytes"] / el / 1e9, 3), "unit": "GB/s", "steps": a.steps,
                "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak", "dtype": "u8",
                "data": "synthetic (device-generated splitmix64 blob)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "blob_bytes": p["blob_bytes"],
                           "piece_length": p["piece_length"], "knobs": "none (KRK_ environment removed)"},
                "defaults": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in p.items()},
                "criteria": {"c1_within_1.2x_one_sha_thread": p["c1_ratio_to_host_sha"] <= 1.2,
                             "stream_at_least_one_crc_thread": p["stream_GBps"] >= p["host_crc_1thread_GBps"]}})


def drop_cache(paths):
    """Evict every file's pages from the page cache (posix_fadvise DONTNEED; the files were
    fsync'ed when written, so their pages are clean and can go)."""
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        try:
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def resident_fraction(paths):
    """Share of the files' pages in the page cache (mincore over a read-only mapping)."""
    import ctypes as C
    libc = C.CDLL(None, use_errno=True)
    libc.mmap.restype = C.c_void_p
    libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
    libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
    libc.mincore.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
    pages = res = 0
    for p in paths:
        n = os.path.getsize(p)
        if not n:
            continue
        fd = os.open(p, os.O_RDONLY)
        try:
            addr = libc.mmap(None, n, 1, 1, fd, 0)  # PROT_READ, MAP_SHARED
            if addr in (None, C.c_void_p(-1).value):
                continue
            k = (n + 4095) // 4096
            vec = (C.c_ubyte * k)()
            if libc.mincore(addr, n, vec) == 0:
                pages += k
                res += sum(v & 1 for v in vec)
            libc.munmap(addr, n)
        finally:
            os.close(fd)
    return res / pages if pages else 0.0


def disk_read_rate(paths, threads=16, chunk=8 << 20):
    """GB/s of plain large reads of the files (no compute), `threads` at a time: the disk
    roofline of the cold leg."""
    from concurrent.futures import ThreadPoolExecutor

    def rd(p):
        buf = bytearray(chunk)
        mv = memoryview(buf)
        got = 0
        with open(p, "rb", buffering=0) as f:
            while True:
                k = f.readinto(mv)
                if not k:
                    return got
                got += k
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(rd, paths))
    return total / (time.perf_counter() - t0) / 1e9, total


def files_cold_leg(a, D, T, rank, world, P):
    """f3 (upload verify + metainfo from the files themselves) on DISK, not
    page cache.  >= a.cold_gib GiB of DISTINCT files (the C3 length law / 64, every file its
    own synthetic content), fsync'ed, and the page cache dropped for every file before every
    pass (posix_fadvise DONTNEED; the resident share measured by mincore).  Passes: the
    library's GPU-only path (offload off) and its default (AUTO offload) -- both read a cold
    batch O_DIRECT through Linux AIO by default -- the page-cache reads (KRK_FILE_DIRECT=0),
    O_DIRECT by synchronous preads (KRK_FILE_AIO=0), fewer live files (KRK_LIVE_CAP=2048), plain reads of the files on 16 threads (the disk roofline), and the
    reference's two reads on the CPU (origin/blobserver/uploader.go:74-94 digest, then
    lib/metainfogen/generator.go:41-58 piece sums): per file back to back (the second read
    from the page cache the first filled, as on an origin with memory to spare) and the two
    passes over the whole set with the cache dropped between them (both reads from disk).
    Every pass's digests and sums are compared; sampled files against the oracle."""
    import shutil
    import tempfile
    from kraken_amd.windowed import c3_lengths
    d = tempfile.mkdtemp(prefix=f"krk_cold_r{rank}_")
    try:
        free = shutil.disk_usage(d).free
        want = min(int(a.cold_gib * (1 << 30)), int(0.6 * free / max(1, world)))
        law = c3_lengths(200_000, scale=64)
        lens, tot = [], 0
        for L in law:
            if tot >= want:
                break
            lens.append(L)
            tot += L
        n = len(lens)
        ids = [(4 << 40) + rank * 1_000_000 + i for i in range(n)]
        top = max(lens)
        buf = D.DeviceBuffer(top)
        pin = D.PinnedArray((top,), np.uint8)
        paths = []
        t_w = time.perf_counter()
        for i, L in enumerate(lens):
            D.check(D.lib.krk_synth_fill_dev(buf.ptr, ids[i], 0, L, 0, None))
            D.synchronize()
            pin.fill_from(buf)
            p = os.path.join(d, f"c{i}")
            fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            try:
                mv = memoryview(pin.a)[:L]
                off = 0
                while off < L:
                    off += os.write(fd, mv[off:])
                os.fsync(fd)
            finally:
                os.close(fd)
            paths.append(p)
        t_w = time.perf_counter() - t_w
        buf.free()
        del pin
        legs = {}

        def leg(name, fn):
            drop_cache(paths)
            cold = resident_fraction(paths[::max(1, n // 64)])
            T.barrier()
            c0, t0 = cpu_seconds(), time.perf_counter()
            out = fn()
            el = T.max_over_ranks(time.perf_counter() - t0)
            cpu = cpu_seconds() - c0
            legs[name] = {"GBps": round(world * tot / el / 1e9, 3), "seconds": round(el, 3),
                          "resident_before": round(cold, 4), "host_cpu_s_per_GB": round(cpu / (tot / 1e9), 4)}
            if name != "disk_read":  # the window loop's split: fill = the reads
                wl = D.windows_last_call()
                legs[name].update({"phases_s": wl["phases_s"], "direct_reads": wl["direct_reads"],
                                   "fill_GBps": round(tot / max(wl["phases_s"]["fill"], 1e-9) / 1e9, 3)})
            return out

        D.set_sha_host_offload(0)
        s_g, d_g = leg("gpu_only", lambda: D.metainfo_digest_files(paths, lens, P))
        legs["gpu_only"].update({k: v for k, v in D.windows_last_call().items()
                                 if k in ("windows", "max_live", "resident_sample")})
        D.set_sha_host_offload(-1)
        try:
            s_a, d_a = leg("default", lambda: D.metainfo_digest_files(paths, lens, P))
            wl = D.windows_last_call()
            legs["default"].update({"host_blobs": wl["host_blobs"], "resident_sample": wl["resident_sample"],
                                    "direct_reads": wl["direct_reads"]})
        finally:
            D.set_sha_host_offload(0)
        # the reads' forms: page cache (the default when cached), O_DIRECT by synchronous
        # preads (the round-4 O_DIRECT path); the default for a cold batch is O_DIRECT through
        # Linux AIO (gpu_only / default above)
        os.environ["KRK_FILE_DIRECT"] = "0"
        try:
            s_d, d_d = leg("page_cache", lambda: D.metainfo_digest_files(paths, lens, P))
        finally:
            os.environ.pop("KRK_FILE_DIRECT", None)
        os.environ["KRK_FILE_DIRECT"], os.environ["KRK_FILE_AIO"] = "1", "0"
        try:
            s_s, d_s = leg("o_direct_sync_preads", lambda: D.metainfo_digest_files(paths, lens, P))
        finally:
            os.environ.pop("KRK_FILE_DIRECT", None)
            os.environ.pop("KRK_FILE_AIO", None)
        # fewer live files: bigger reads per file per window (512 MiB / live), page cache
        os.environ["KRK_LIVE_CAP"], os.environ["KRK_FILE_DIRECT"] = "2048", "0"
        try:
            s_l, d_l = leg("gpu_only_live2048", lambda: D.metainfo_digest_files(paths, lens, P))
            legs["gpu_only_live2048"]["max_live"] = D.windows_last_call()["max_live"]
        finally:
            os.environ.pop("KRK_LIVE_CAP", None)
            os.environ.pop("KRK_FILE_DIRECT", None)
        # fewer live files read O_DIRECT: larger disk requests (a window holds one chunk of
        # every live file; 512 MiB / live a chunk)
        for cap in (a.cold_live_caps or []):
            os.environ["KRK_LIVE_CAP"], os.environ["KRK_FILE_DIRECT"] = str(cap), "1"
            try:
                nm = f"gpu_only_live{cap}_direct"
                s_x, d_x = leg(nm, lambda: D.metainfo_digest_files(paths, lens, P))
                legs[nm]["max_live"] = D.windows_last_call()["max_live"]
                legs[nm]["outputs_equal_gpu_only"] = bool(np.array_equal(d_x, d_g) and all(
                    np.array_equal(x, y) for x, y in zip(s_x, s_g)))
            finally:
                os.environ.pop("KRK_LIVE_CAP", None)
                os.environ.pop("KRK_FILE_DIRECT", None)
        rate, got = leg("disk_read", lambda: disk_read_rate(paths))
        # the first leg again, last (the first pass after writing the files runs slow on some
        # boxes): the order effect beside the paths' differences
        D.set_sha_host_offload(0)
        s_r, d_r = leg("gpu_only_again", lambda: D.metainfo_digest_files(paths, lens, P))
        legs["disk_read"]["what"] = "plain 8 MiB reads of every file on 16 threads, no compute (the disk roofline)"
        same = all(np.array_equal(d_g, y) for y in (d_a, d_d, d_l, d_s, d_r)) and all(
            all(np.array_equal(x, y) for y in ys) for x, *ys in zip(s_g, s_a, s_d, s_l, s_s, s_r))
        from oracle import oracle as O  # checker and CPU baseline only
        O.build()
        import hashlib
        ok = True
        for i in sorted({0, n // 2, n - 1, int(np.argmax(lens))}):
            x = O.synth(ids[i], lens[i])
            ok = ok and bytes(d_g[i]) == hashlib.sha256(x.tobytes()).digest() and np.array_equal(
                s_g[i], O.calc_piece_sums(x, P)[1])
        cpu = None
        if rank == 0 and not a.no_cpu_baseline:
            drop_cache(paths)
            t_c, s_c, off_c, dg_c = O.baseline_files(paths, lens, P, node_cores(), passes=3)
            drop_cache(paths)
            t_1 = O.baseline_files(paths, lens, P, node_cores(), passes=1)[0]
            drop_cache(paths)
            t_2 = O.baseline_files(paths, lens, P, node_cores(), passes=2)[0]
            same_c = bool(np.array_equal(dg_c, d_g)) and all(
                np.array_equal(s_c[int(off_c[i]):int(off_c[i + 1])], s_g[i]) for i in range(n))
            cpu = {"value": round(tot / t_c / 1e9, 3), "unit": "GB/s", "cores": node_cores(),
                   "cores_source": CORES_SOURCE, "kind": "port", "seconds": round(t_c, 3),
                   "two_disk_reads_GBps": round(tot / (t_1 + t_2) / 1e9, 3),
                   "two_disk_reads_seconds": [round(t_1, 3), round(t_2, 3)], "outputs_match_gpu": same_c,
                   "sample": f"all {n} cold files: Digester.FromReader then calcPieceSums over each file, 32 KiB "
                             "reads, SHA-NI and PCLMUL, one file per thread (oracle/oracle.c orc_baseline_files); "
                             "value = the two reads back to back per file (the second from the page cache), "
                             "two_disk_reads = the two passes over the set with the cache dropped between"}
        return {"files": n, "bytes": tot, "GiB": round(tot / (1 << 30), 2), "dir_free_GB": round(free / 1e9, 1),
                "write_s": round(t_w, 2), "legs": legs, "outputs_equal": bool(same), "sampled_equal_oracle": bool(ok),
                "cpu_baseline": cpu,
                "roofline": {"bound": "disk", "peak": legs["disk_read"]["GBps"], "unit": "GB/s",
                             "achieved": legs["gpu_only"]["GBps"],
                             "frac": round(legs["gpu_only"]["GBps"] / max(legs["disk_read"]["GBps"], 1e-9), 4)}}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_engine(a, D, T, rank, world, res):
    """The submission engine under concurrent Digesters: tests/native/digesters
    runs warmup + steps rounds of 256 GPU-placed digesters (a round = every digester's 16 MiB
    and its digest); value = the timed rounds' bytes over their summed seconds.  Every digest
    is checked against the host SHA-256 of the same bytes in the child (digests_match).  The
    rate lives here, not in the parity tests.  Then (unless --no-sweep)
    the crossover sweep of VERDICT r04 item 4: N concurrent digesters on each placement."""
    exe = os.path.join(ROOT, "tests", "native", "digesters")
    n, mib = 256, 16
    r = subprocess.run([exe, str(n), str(mib), str(a.warmup + a.steps)], capture_output=True, text=True, timeout=900)
    rounds = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or len(rounds) != a.warmup + a.steps:
        raise SystemExit(f"bench.py: digesters failed (rc {r.returncode}): {r.stderr[-2000:]}")
    timed = rounds[a.warmup:]
    secs = sum(x["seconds"] for x in timed)
    el = T.timed_region(secs)
    total = n * (mib << 20) * len(timed)
    res.update({"metric": "concurrent GPU Digester GB/s (256 uploads)", "value": round(world * total / el / 1e9, 3),
                "unit": "GB/s", "steps": a.steps, "ms_per_step": round(el / a.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "dtype": "u8",
                "data": "synthetic (seeded random bytes, host memory of the native caller)",
                "config": {"workload": WORKLOADS[a.workload]["desc"], "digesters": n, "bytes_each": mib << 20,
                           "placement": "KRK_PLACE_GPU (the submission engine)"},
                "rounds": [{k: x[k] for k in ("round", "seconds", "GBps", "MBps_per_stream", "sha_launches",
                                              "streams_per_launch", "digests_match")} for x in rounds],
                "digests_match": all(x["digests_match"] for x in rounds),
                "per_stream_ceiling_MBps": "~59 (the eight-lane batch kernel, DESIGN.md 4.2): 256 x 59 MB/s = "
                                           "15.1 GB/s"})
    if not a.no_sweep:
        res["crossover"] = digester_crossover_sweep(exe, mib)


ENGINE_SWEEP = (256, 640, 1024, 2048, 4096)


def digester_crossover_sweep(exe, mib, sizes=ENGINE_SWEEP, threads=256):
    """N concurrent Digesters (one per upload / cache fill,
    origin/blobserver/uploader.go:75, lib/store/ca_store.go:119) driven from `threads` native
    threads (each owns N / threads digesters and writes them round-robin), on the GPU engine
    and on the host (SHA-NI on the writers' threads under the CPU tokens): aggregate GB/s and
    per-stream MB/s, the measured crossover (linear interpolation of the first N where the GPU
    overtakes), and AUTO's switch point from the planner rates (krk_digester_host_streams)."""
    import ctypes as C
    from kraken_amd._capi import check, lib
    rows = []
    for m in sizes:
        row = {"digesters": m, "threads": min(m, threads)}
        for pl in ("gpu", "host", "auto"):
            r = subprocess.run([exe, str(m), str(mib), "4", str(1 << 20), pl, str(threads)], capture_output=True,
                               text=True, timeout=900)
            rr = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or len(rr) != 4:
                raise SystemExit(f"bench.py: digesters {m} {pl} failed (rc {r.returncode}): {r.stderr[-2000:]}")
            # rounds 1-3 (round 0 grows the slot pool): the median round
            x = sorted(rr[1:], key=lambda q: q["GBps"])[1]
            row[pl] = {"GBps": x["GBps"], "rounds_GBps": [q["GBps"] for q in rr[1:]],
                       "MBps_per_stream": x["MBps_per_stream"], "on_gpu": x["on_gpu"],
                       "sha_launches": x["sha_launches"], "streams_per_launch": x["streams_per_launch"],
                       "pinned_bytes": x["pinned_bytes"], "digests_match": x["digests_match"]}
        rows.append(row)
    cross = None
    for lo, hi in zip(rows, rows[1:]):
        d_lo = lo["gpu"]["GBps"] - lo["host"]["GBps"]
        d_hi = hi["gpu"]["GBps"] - hi["host"]["GBps"]
        if d_lo <= 0 < d_hi:
            cross = lo["digesters"] + (hi["digesters"] - lo["digesters"]) * (-d_lo) / (d_hi - d_lo)
            break
    if cross is None and rows and rows[0]["gpu"]["GBps"] > rows[0]["host"]["GBps"]:
        cross = float(rows[0]["digesters"])  # the GPU already wins at the smallest N
    auto = C.c_int64()
    check(lib.krk_digester_host_streams(C.byref(auto)))
    a_n = auto.value if auto.value < (1 << 62) else None
    within = (a_n is not None and cross is not None and abs(a_n + 1 - cross) <= 0.2 * cross) or \
        (a_n is None and cross is None)
    return {"rows": rows, "measured_crossover": None if cross is None else round(cross, 1),
            "engine_slot_src": os.environ.get("KRK_ENGINE_SLOT_SRC", "zerocopy"),
            "auto_host_streams": a_n, "auto_within_20pct": bool(within),
            "rates": D_rates_brief(),
            "what": f"{mib} MiB a digester, writes of 1 B - 1 MiB, {threads} native threads (tests/native/digesters), "
                    "median of 3 rounds after a warm one; gpu / host: every digester on that placement, auto: the "
                    "library's default (the first auto_host_streams live ones on the host, the rest on the GPU); "
                    "measured_crossover: N where the GPU engine's aggregate overtakes the host's (interpolated); "
                    "auto_host_streams: krk_digester_host_streams, AUTO keeps digesters on the host up to it"}


def D_rates_brief():
    from kraken_amd import device as D
    r = D.planner_rates()
    return {"sha_stream_MBps": [round(x / 1e6, 2) for x in r["sha_stream_bps"]], "h2d_GBps": round(r["h2d_bps"] / 1e9, 2),
            "host_sha_GBps_per_thread": round(r["host_sha_bps"] / 1e9, 3), "source": r["source"],
            "host_cpus": host_cores()}


def visible_devices() -> int:
    """gfx950 devices a rank would see, counted in a child process so that the parent
    (which only spawns and waits) never initialises the GPU itself."""
    r = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); "
                        "from kraken_amd import device as D; print(D.device_count())" % ROOT],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, devices=None, rehearse=False, script=None):
    """`bench.py --gpus N` without a launcher: start N rank processes of this same
    command (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env, as
    torch.distributed.run would set them) and wait for them; rank 0 prints the line.
    Fewer than N visible devices is an error unless `rehearse` (ranks then share the
    visible devices round-robin and the line says so).  Returns the exit code: 0 only
    if every rank exited 0; a failed rank ends the others."""
    if devices is None:
        devices = visible_devices()
    if devices < n and not rehearse:
        print(f"bench.py: --gpus {n} but {devices} gfx950 device(s) visible; pass --rehearse to run {n} ranks "
              f"on {devices} device(s)", file=sys.stderr, flush=True)
        return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KRK_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # the exact processes this call started
                    q.kill()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); without a launcher's WORLD_SIZE, N rank processes are spawned")
    ap.add_argument("--rehearse", action="store_true",
                    help="allow --gpus N on fewer than N devices (ranks share devices; the line says so)")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 3; C5: 50)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 1; C5: 5)")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--blobs", type=int, default=0, help="override the blob (or digest) count")
    ap.add_argument("--nodes", type=int, default=16, help="C5: origins in the ring")
    ap.add_argument("--window-gib", type=int, default=48, help="C3: device window size")
    ap.add_argument("--live-cap", type=int, default=0, help="C3: live streams per window (0 = the planner's)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="C3: run rank 0's LPT shard of an N-GPU run on this GPU (no collective exists to emulate)")
    ap.add_argument("--emulate-rank", type=int, default=None,
                    help="C3 with --emulate-world: run this rank's shard instead of rank 0's (every shard in turn "
                         "gives the emulated job's max over ranks)")
    ap.add_argument("--no-admission", action="store_true",
                    help="C3: all blobs live from window 0 (no longest-first admission under the two-lane cap)")
    ap.add_argument("--host-lane", action="store_true",
                    help="C3: also run the batch with the host lane (the longest blobs hashed on host threads "
                         "while the windows run the rest), reported as host_offload beside the GPU-only value")
    ap.add_argument("--host-lane-k", type=int, default=-1, help="C3: blobs the host lane takes (-1 = the planner's)")
    ap.add_argument("--tail-handoff", action="store_true",
                    help="C3: also run the batch with the tail handoff (host threads steal the chains with the most "
                         "bytes left at window boundaries), reported as tail_handoff beside the GPU-only value")
    ap.add_argument("--tail-threads", type=int, default=0, help="C3 tail handoff: host threads (0 = the CPU budget - 1)")
    ap.add_argument("--cold-live-caps", type=int, nargs="*", default=None,
                    help="files workload: extra cold legs read O_DIRECT with these live-file caps")
    ap.add_argument("--tail-ring", type=int, default=0, help="C3 tail handoff: device pieces a thread keeps in flight")
    ap.add_argument("--tail-crc-beside-sha", action="store_true",
                    help="C3 tail handoff: each window's CRC launch beside its SHA launch (A/B; default: beside "
                         "only when the windows are full)")
    ap.add_argument("--tail-piece-mib", type=int, default=0, help="C3 tail handoff: MiB a device piece")
    ap.add_argument("--c3-tail-only", action="store_true",
                    help="C3: skip the GPU-only windows (measurement runs of the tail handoff; no value line)")
    ap.add_argument("--hrw-int32", action="store_true", help="C5: int32 owner indices even for <= 255 nodes")
    ap.add_argument("--regen-serial", action="store_true",
                    help="c5regen: piece sums then InfoHashes (no krk_metainfo_batch_dev pipelining)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--pmc-json", default=None, help="PMC traffic JSON (default: the newest committed for the workload)")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the live SHA issue-ceiling run (profiler passes: keeps its launches out of the trace)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host buffers, PCIe) leg")
    ap.add_argument("--no-offload", action="store_true",
                    help="C1 / c5regen_digest: skip the SHA-256 host-offload leg")
    ap.add_argument("--no-sweep", action="store_true", help="C5: skip the N x MaxReplica x healthy grid")
    ap.add_argument("--e2e-mb", type=int, default=100, help="bytes per blob for the end-to-end leg (MiB; C2: 100)")
    ap.add_argument("--cold-gib", type=float, default=32.0,
                    help="files: GiB of distinct files for the cold (page cache dropped) leg; 0 = skip it")
    ap.add_argument("--e2e-only", action="store_true",
                    help="C2: only the end-to-end leg (profiler passes of the host path)")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = WORKLOADS[a.workload].get("steps", 3)
    if a.warmup is None:
        a.warmup = WORKLOADS[a.workload].get("warmup", 1)

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:], rehearse=a.rehearse))
    rank, world, local = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1), _env_int("LOCAL_RANK", 0)
    if world != a.gpus and "WORLD_SIZE" in os.environ:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist  # control-plane barrier/max only; no data-path collective
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from kraken_amd import device as D

    # one process per GPU; a --rehearse run shares the visible devices round-robin
    ndev = D.device_count()
    if world > ndev and not a.rehearse:
        raise SystemExit(f"bench.py: {world} ranks but {ndev} gfx950 device(s) visible (pass --rehearse to share)")
    a.device = local % max(1, ndev)
    D.set_device(a.device)
    # `value` is the GPU-only path (every chain on the device): the library's default
    # (planner-gated host offload, AUTO) is measured beside it as `host_offload` /
    # end_to_end.host_hybrid
    D.set_sha_host_offload(0)
    T = Timer(D, dist)
    res = {"n_gpus": world, "warmup": a.warmup, "vs_baseline": None}
    if world > ndev:
        res["rehearsal"] = f"{world} ranks on {ndev} device(s): not an N-GPU measurement"
    kind = WORKLOADS[a.workload]["kind"]
    {"metainfo": run_metainfo, "pieces": run_pieces, "chunked": run_chunked, "hrw": run_hrw, "regen": run_regen,
     "verify": run_verify, "engine": run_engine, "files": run_files, "defaults": run_defaults}[kind](
        a, D, T, rank, world, res)
    # rank 0's CPU baseline (if any) ran after the timed region, behind this barrier the
    # other ranks wait at; then every rank's device and time go into the line, so an N-GPU
    # line shows it ran on N distinct GPUs
    T.barrier()
    devs = T.gather(D.device_pci_bus_id())
    cpus, node, src = host_budget()
    res["host_budget"] = {"rank_cpus": T.gather(cpus), "node_cpus": node, "source": src,
                          "local_world_size": _env_int("LOCAL_WORLD_SIZE", 1),
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    if world > 1 or T.rank_s:
        res["rank_devices"] = devs
        if T.rank_s:
            res["rank_ms"] = [round(x * 1e3, 3) for x in T.rank_s]
        if world > 1 and len(set(devs)) < world and "rehearsal" not in res:
            raise SystemExit(f"bench.py: {world} ranks on {len(set(devs))} distinct device(s): {devs}")
    order = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config"]
    line = {k: res[k] for k in order if k in res}
    line.update({k: v for k, v in res.items() if k not in line})
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
