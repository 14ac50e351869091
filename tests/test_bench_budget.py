"""VERDICT r04 item 1 (CPU, gloo): an N-rank bench line under a launcher's environment.

torch.distributed.run sets OMP_NUM_THREADS=1 for every rank of a multi-rank node and
LOCAL_WORLD_SIZE to the ranks on the node.  The ranks here run bench.main() for real
(gloo barrier, max-over-ranks timing, rank 0's cpu_baseline on the oracle), with a stub
device module standing in for kraken_amd.device (no GPU in this container); the host
budget they report comes from the real library (krk_host_cpu_budget).  Asserted:
  * each rank's library budget is the node's CPUs / LOCAL_WORLD_SIZE, not 1;
  * rank 0's cpu_baseline runs on all of the node's cores (GOMAXPROCS = every core).
tests/test_gpu_bench_contract.py asserts the same on the GPU box with the real device."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from kraken_amd import _capi  # noqa: E402

STUB_RANK = r'''
import hashlib, os, sys, types
import numpy as np
root, out = sys.argv[1], sys.argv[2]
sys.path.insert(0, root)
import kraken_amd
from oracle import oracle as O   # the stub device's outputs (test infrastructure)

D = types.ModuleType("kraken_amd.device")

class _Buf:
    def __init__(self, n):
        self.a = np.zeros(max(n, 1), np.uint8)

class BlobArena:
    def __init__(self, lengths, piece_length, blob_ids=None):
        self.lengths = np.asarray(lengths, np.uint64)
        self.P = int(piece_length)
        self.ids = list(blob_ids)
        self.n_pieces = np.array([-(-int(L) // self.P) for L in self.lengths], np.uint64)
        self.sums_off = np.zeros(len(self.lengths), np.uint64)
        self.sums_off[1:] = np.cumsum(self.n_pieces)[:-1]
        self.total_pieces = int(self.n_pieces.sum())

class BatchOutputs:
    def __init__(self, arena):
        self.sums = _Buf(arena.total_pieces * 4)
        self.digests = _Buf(len(arena.lengths) * 32)

class PinnedArray:
    def __init__(self, shape, dtype):
        self.a = np.zeros(shape, dtype)
    def fill_from(self, dev, offset=0):
        self.a.view(np.uint8).reshape(-1)[:] = dev.a[offset:offset + self.a.nbytes]
        return self.a

def metainfo_digest(arena, out, stream=None):
    for i, (b, L) in enumerate(zip(arena.ids, arena.lengths)):
        data = O.synth(int(b), int(L))
        out.digests.a[32 * i:32 * i + 32] = np.frombuffer(hashlib.sha256(data.tobytes()).digest(), np.uint8)
        s = np.asarray(O.calc_piece_sums(data, arena.P)[1], np.uint32)
        o = int(arena.sums_off[i]) * 4
        out.sums.a[o:o + s.nbytes] = s.view(np.uint8)

class KernelTimer:
    def __enter__(self):
        return self
    def __exit__(self, *a):
        pass
    @staticmethod
    def stats(kernel):
        return (1, 2.0 if kernel == "sha256_multi" else 1.0)

D.BlobArena, D.BatchOutputs, D.PinnedArray, D.KernelTimer = BlobArena, BatchOutputs, PinnedArray, KernelTimer
D.metainfo_digest = metainfo_digest
D.device_count = lambda: 1
D.set_device = lambda d: None
D.set_sha_host_offload = lambda t: None
D.synchronize = lambda: None
D.sha_lanes_per_stream = lambda n: 8
D.device_pci_bus_id = lambda: "0000:00:00.0"
sys.modules["kraken_amd.device"] = D
kraken_amd.device = D

import bench
rank = os.environ["RANK"]
with open(os.path.join(out, "budget%s.txt" % rank), "w") as f:
    f.write("%d %d %s" % bench.host_budget())
sys.argv = ["bench.py"] + sys.argv[3:]
stdout = sys.stdout
with open(os.path.join(out, "line%s.txt" % rank), "w") as f:
    sys.stdout = f
    try:
        bench.main()
    finally:
        sys.stdout = stdout
'''


@pytest.mark.timeout(300)
def test_launcher_env_budget_and_baseline_cores(tmp_path, monkeypatch):
    node = _capi.host_cpu_budget()[1]
    world = 4
    script = tmp_path / "stub_rank.py"
    script.write_text(STUB_RANK)
    # a torch.distributed.run-shaped environment: OMP_NUM_THREADS=1 a rank
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    monkeypatch.delenv("KRK_HOST_CPUS", raising=False)
    args = [ROOT, str(tmp_path), "--gpus", str(world), "--rehearse", "--workload", "small", "--blobs", str(node),
            "--steps", "1", "--warmup", "0", "--cpu-seconds", "0.2", "--no-e2e", "--no-ceiling"]
    assert bench.spawn_ranks(world, args, devices=1, rehearse=True, script=str(script)) == 0
    want = max(1, node // world)
    for r in range(world):
        cpus, nd, src = (tmp_path / f"budget{r}.txt").read_text().split()
        assert (int(cpus), int(nd), src) == (want, node, "node/LOCAL_WORLD_SIZE")
    lines = [l for l in (tmp_path / "line0.txt").read_text().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and "rehearsal" in d
    hb = d["host_budget"]
    assert hb["rank_cpus"] == [want] * world and hb["node_cpus"] == node
    assert hb["source"] == "node/LOCAL_WORLD_SIZE" and hb["local_world_size"] == world
    assert hb["omp_num_threads"] == "1"
    cb = d["cpu_baseline"]
    assert cb["cores"] == node and "cgroup" in cb["cores_source"]
    assert cb["outputs_match_gpu"] is True
    for r in range(1, world):  # only rank 0 prints
        assert not [l for l in (tmp_path / f"line{r}.txt").read_text().splitlines() if l.startswith("{")]


def test_budget_sources(tmp_path):
    """The library's per-process budget under each environment (fresh processes: it is
    read once)."""
    import subprocess
    node = _capi.host_cpu_budget()[1]
    code = "from kraken_amd import _capi; print(*_capi.host_cpu_budget())"
    base = {k: v for k, v in os.environ.items() if k not in ("OMP_NUM_THREADS", "LOCAL_WORLD_SIZE", "KRK_HOST_CPUS")}
    cases = [({}, (node, node, "node")),
             ({"LOCAL_WORLD_SIZE": "4", "OMP_NUM_THREADS": "1"}, (max(1, node // 4), node, "node/LOCAL_WORLD_SIZE")),
             ({"LOCAL_WORLD_SIZE": "1", "OMP_NUM_THREADS": "2"}, (min(2, node), node,
                                                                   "OMP_NUM_THREADS" if node > 2 else "node")),
             ({"KRK_HOST_CPUS": "3", "LOCAL_WORLD_SIZE": "8"}, (3, node, "KRK_HOST_CPUS")),
             ({"LOCAL_WORLD_SIZE": str(4 * node)}, (1, node, "node/LOCAL_WORLD_SIZE"))]
    for env, want in cases:
        r = subprocess.run([sys.executable, "-c", code], env=dict(base, **env), capture_output=True, text=True,
                           cwd=ROOT, timeout=60)
        assert r.returncode == 0, r.stderr
        c, n, s = r.stdout.split()
        assert (int(c), int(n), s) == want, (env, r.stdout)
