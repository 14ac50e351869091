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
