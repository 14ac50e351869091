"""bench.py --gpus N without a launcher (CPU): the parent spawns N rank processes with
torch.distributed.run's environment, refuses to run N ranks on fewer devices unless
--rehearse, and fails when a rank fails.  The rank body here is a stand-in script
(no GPU in this container); tests/test_gpu_bench_contract.py runs the real one."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = r'''
import json, os, sys
out = sys.argv[1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "KRK_BENCH_SPAWNED")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]}, f)
sys.exit(int(os.environ["RANK"]) == int(os.environ.get("FAIL_RANK", "-1")) and 3 or 0)
'''


@pytest.fixture
def child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_spawns_n_ranks_with_launcher_env(child, tmp_path):
    rc = bench.spawn_ranks(4, [str(tmp_path), "--gpus", "4"], devices=4, script=child)
    assert rc == 0
    seen = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    assert [s["RANK"] for s in seen] == ["0", "1", "2", "3"]
    assert all(s["WORLD_SIZE"] == "4" and s["MASTER_ADDR"] == "127.0.0.1" for s in seen)
    assert len({s["MASTER_PORT"] for s in seen}) == 1 and all(s["KRK_BENCH_SPAWNED"] == "1" for s in seen)
    assert all(s["argv"] == [str(tmp_path), "--gpus", "4"] for s in seen)


def test_fewer_devices_refused_unless_rehearse(child, tmp_path):
    assert bench.spawn_ranks(2, [str(tmp_path)], devices=1, script=child) == 2
    assert not list(tmp_path.glob("rank*.json"))
    assert bench.spawn_ranks(2, [str(tmp_path)], devices=1, rehearse=True, script=child) == 0
    assert len(list(tmp_path.glob("rank*.json"))) == 2


def test_failed_rank_fails_the_run(child, tmp_path, monkeypatch):
    monkeypatch.setenv("FAIL_RANK", "1")
    assert bench.spawn_ranks(2, [str(tmp_path)], devices=2, script=child) == 3


TIMER_CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[2])
import torch.distributed as dist
import bench
dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
T = bench.Timer(None, dist)
r = int(os.environ["RANK"])
mx = T.timed_region(0.5 + r)
devs = T.gather("0000:%02x:00.0" % (r + 3))
with open(os.path.join(sys.argv[1], "t%d.json" % r), "w") as f:
    json.dump({"max": mx, "rank_s": T.rank_s, "devs": devs}, f)
dist.destroy_process_group()
'''


def test_timer_gathers_every_ranks_time_and_device(tmp_path):
    """VERDICT r03 item 4 (CPU, gloo, world 2): the timed region's max over ranks, every
    rank's own time and every rank's device id reach every rank (rank 0 prints them as
    rank_ms / rank_devices)."""
    script = tmp_path / "timer_child.py"
    script.write_text(TIMER_CHILD)
    assert bench.spawn_ranks(2, [str(tmp_path), ROOT], devices=2, script=str(script)) == 0
    for r in range(2):
        d = json.load(open(tmp_path / f"t{r}.json"))
        assert d["max"] == 1.5 and d["rank_s"] == [0.5, 1.5]
        assert d["devs"] == ["0000:03:00.0", "0000:04:00.0"]
