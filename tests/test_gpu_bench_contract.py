"""bench.py's one-line JSON contract (the driver parses it at every round end), on a
small workload: required keys and types, the roofline and cpu_baseline objects, and
the CPU baseline's outputs equal to the GPU's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line_contract(gpu):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "small", "--steps", "2",
                        "--warmup", "1", "--cpu-seconds", "1", "--e2e-mb", "4"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k, t in [("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int), ("warmup", int),
                 ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str), ("dtype", str),
                 ("data", str), ("config", dict)]:
        assert isinstance(d[k], t), k
    assert d["vs_baseline"] is None and d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert "workload" in d["config"]
    roof = d["roofline"]
    assert roof["bound"] in ("hbm", "mfma", "valu") and roof["unit"] == "GB/s"
    assert roof["peak"] == 8000.0 if roof["bound"] == "hbm" else roof["hbm"]["peak"] == 8000.0
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["outputs_match_gpu"] is True


def test_bench_gpus_2_spawns_two_ranks(gpu):
    """`bench.py --gpus 2` with no launcher spawns two rank processes (here sharing the
    one GPU: --rehearse) and reports the whole job: n_gpus == 2 and value == both
    ranks' bytes over the max-over-ranks time.  VERDICT r03 item 4: the N-rank line is
    self-verifying -- rank 0's CPU baseline (timed after the GPU region while the other
    ranks wait), every rank's device PCI bus id and own time; here both ranks share the
    one GPU, which only a rehearsal may."""
    env = dict(os.environ, OMP_NUM_THREADS="1")  # what torch.distributed.run gives each rank of a node
    env.pop("KRK_HOST_CPUS", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse", "--blobs", "20",
                        "--steps", "1", "--warmup", "1", "--cpu-seconds", "1", "--no-e2e", "--no-ceiling"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and "rehearsal" in d
    assert d["config"]["blobs_per_gpu"] == 20 and d["config"]["parallelism"].startswith("blob-sharded x2")
    want = 2 * d["config"]["bytes_per_gpu"] * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3) / 1e9
    assert abs(d["value"] - want) / want < 1e-3, (d["value"], want)
    assert len(d["rank_devices"]) == 2 and len(set(d["rank_devices"])) == 1  # one GPU, two ranks
    assert len(d["rank_ms"]) == 2 and abs(max(d["rank_ms"]) - d["ms_per_step"] * d["steps"]) < 1e-2
    cb = d["cpu_baseline"]
    assert cb["cores"] >= 1 and cb["value"] > 0 and cb["outputs_match_gpu"] is True
    # each rank's library budget is the node's CPUs / LOCAL_WORLD_SIZE
    # (a launcher's OMP_NUM_THREADS=1 does not shrink it); rank 0's baseline runs on the node
    hb = d["host_budget"]
    node = hb["node_cpus"]
    assert hb["rank_cpus"] == [max(1, node // 2)] * 2 and hb["source"] == "node/LOCAL_WORLD_SIZE", hb
    assert cb["cores"] == min(node, 20), (cb["cores"], node)


def test_bench_gpus_more_than_visible_refused(gpu):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpu.device_count() + 1),
                        "--blobs", "2", "--steps", "1", "--no-cpu-baseline", "--no-e2e"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0 and "--rehearse" in r.stderr and not r.stdout.strip()
