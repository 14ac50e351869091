"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 control plane: LPT
blob sharding and the host gather of per-blob results.  The per-blob compute here
is the CPU oracle (no GPU in this suite); tests/test_gpu_shard_gloo.py runs the same
sharding and gather with the product (the C ABI on the GPU) as the compute."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kraken_amd.shard import gather_results, lpt_shard, shard_loads


def test_lpt_balance():
    rng = np.random.default_rng(0)
    lens = 104857600 + rng.integers(0, 968884225, size=2000)  # config C3 size law
    for world in (1, 2, 4, 8):
        shards = lpt_shard(lens, world)
        assert sorted(i for s in shards for i in s) == list(range(len(lens)))
        loads = shard_loads(lens, shards)
        assert max(loads) - min(loads) <= int(lens.max())  # LPT bound
        assert max(loads) / (sum(loads) / world) < 1.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lens, piece, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    mine = lpt_shard(lens, world)[rank]
    local = {}
    for i in mine:
        data = O.synth(i, int(lens[i]))
        local[i] = (O.sha256(data).hex(), O.calc_piece_sums(data, piece)[1].tolist())
    merged = gather_results(local, dist)
    if rank == 0:
        q.put(merged)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_gather_world2(orc):
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 200000, size=24)
    piece = 65536
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lens, piece, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(merged) == list(range(len(lens)))
    for i, L in enumerate(lens):
        data = orc.synth(i, int(L))
        assert merged[i][0] == orc.sha256(data).hex()
        assert merged[i][1] == orc.calc_piece_sums(data, piece)[1].tolist()
