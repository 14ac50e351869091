"""The C3 tail handoff run twice (or N times) in one process on rank 0's shard of an emulated
8-GPU run ('Leg order'): does a second heavy leg in the same process lose,
whatever the first was?  One JSON line per run: GB/s for the job, copy waits, twin copy rate."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from kraken_amd import device as D  # noqa: E402
from kraken_amd.shard import lpt_shard  # noqa: E402
from kraken_amd.windowed import TAIL_CHUNK, TailHandoffRun, c3_lengths  # noqa: E402


def main():
    """argv: runs [lane]: 'lane' runs the host-lane leg (WindowedRun with the planner's K
    longest blobs on 15 host threads) first, as bench.py's C3 line once did."""
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    D.set_device(0)
    lens_all = c3_lengths(20000)
    mine = lpt_shard(lens_all, 8)[0]
    ids = [(2 << 40) + int(i) for i in mine]
    lens = [int(lens_all[i]) for i in mine]
    total = int(sum(lens_all))
    if len(sys.argv) > 2 and sys.argv[2] == "lane":
        from kraken_amd.windowed import WindowedRun, host_lane_plan, window_stream_cap
        W = 48 << 30
        k, _, _ = host_lane_plan(D, lens, W, window_stream_cap(D, len(lens)), 15)
        wr = WindowedRun(D, ids, lens, 4 << 20, W, host_lane=(k, 15))
        t0 = time.perf_counter()
        wr.run()
        el = time.perf_counter() - t0
        wr.close()
        print(json.dumps({"run": "host lane", "GBps": round(total / el / 1e9, 2), "blobs_on_host": int(k)}),
              flush=True)
    if len(sys.argv) > 3 and sys.argv[3] == "timeline":  # D2H rate over time after the lane
        import ctypes as C
        import numpy as np
        from pinned_d2h_probe import PIECE, rate
        src = D.DeviceBuffer(PIECE)
        s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(s)))
        bufs = [D.PinnedArray((PIECE,), np.uint8) for _ in range(8)]
        ptrs = [b.ptr for b in bufs]
        rate(ptrs, src, s, reps=1)
        t0 = time.perf_counter()
        line = []
        while time.perf_counter() - t0 < 30:
            line.append((round(time.perf_counter() - t0, 2), round(rate(ptrs, src, s, reps=1), 1)))
            time.sleep(0.25)
        print(json.dumps({"d2h_GBps_timeline_after_lane": line}), flush=True)
    if len(sys.argv) > 3 and sys.argv[3] == "probe":  # the pinned buffers a tail run would get now
        import ctypes as C
        import numpy as np
        from pinned_d2h_probe import PIECE, numa_node, rate
        src = D.DeviceBuffer(PIECE)
        s = C.c_void_p()
        D.check(D.lib.krk_stream_create(C.byref(s)))
        all_cpus = os.sched_getaffinity(0)
        for name, dma, cpus in (("krk_host_alloc_dma", True, None), ("krk_host_alloc", False, None),
                                ("krk_host_alloc from node-1 CPUs", False, set(range(64, 128)) & all_cpus),
                                ("krk_host_alloc_dma from node-1 CPUs", True, set(range(64, 128)) & all_cpus)):
            if cpus:
                os.sched_setaffinity(0, cpus)
            bufs = [D.PinnedArray((PIECE,), np.uint8, dma_target=dma) for _ in range(120)]
            os.sched_setaffinity(0, all_cpus)
            huge = 0
            try:  # the buffers' transparent huge pages (kB), from smaps
                lo, hi = min(b.ptr for b in bufs), max(b.ptr for b in bufs) + PIECE
                cur = None
                for line in open("/proc/self/smaps"):
                    if "-" in line.split()[0] and len(line.split()) > 4:
                        a, b2 = (int(x, 16) for x in line.split()[0].split("-"))
                        cur = lo <= a < hi
                    elif cur and line.startswith("AnonHugePages:"):
                        huge += int(line.split()[1])
            except OSError:
                huge = -1
            ptrs = [b.ptr for b in bufs]
            rate(ptrs, src, s, reps=1)
            per = [round(rate([p], src, s, reps=2), 1) for p in ptrs]
            nodes = [numa_node(p) for p in ptrs]
            print(json.dumps({"probe": name, "huge_pages_GiB": round(huge / (1 << 20), 2),
                              "GBps_min_median_max": [min(per), sorted(per)[60], max(per)],
                              "slow_below_40": sum(x < 40 for x in per),
                              "nodes": {str(n): nodes.count(n) for n in set(nodes)},
                              "slow_by_node": {str(n): sum(1 for x, m in zip(per, nodes) if x < 40 and m == n)
                                               for n in set(nodes)}}), flush=True)
            del bufs
    for r in range(reps):
        tr = TailHandoffRun(D, ids, lens, 4 << 20, min(48 << 30, len(lens) * TAIL_CHUNK), 15)
        t0 = time.perf_counter()
        tr.run()
        el = time.perf_counter() - t0
        st = tr.stats
        tr.close()
        print(json.dumps({"run": r, "GBps": round(total / el / 1e9, 2), "seconds": round(el, 3),
                          "copy_wait_s": st["thread_phases_s"]["copy_wait"], "host_bytes": st["host_bytes"],
                          "twin_copy_GBps": st["twin_copy_GBps_before_run"],
                          "loop_generate_s": st["loop_generate_s"]}), flush=True)


if __name__ == "__main__":
    main()
