"""The N>1 path on the product: two processes (world_size 2, gloo control plane, both
on device 0 of the one-GPU test box) each run their LPT shard of a batch through the
C ABI (krk_metainfo_digest_host: piece sums + SHA-256 on the GPU), and the per-blob
results are gathered to rank 0 on the host -- no data-path collective (SURVEY.md
8(e)).  Rank 0 checks every blob against the oracle."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kraken_amd.shard import gather_results, lpt_shard

pytestmark = pytest.mark.gpu


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
    from kraken_amd import device as D
    from oracle import oracle as O  # the generator of the synthetic blob bytes only
    D.set_device(0)
    mine = lpt_shard(lens, world)[rank]
    datas = [O.synth(i, int(lens[i])) for i in mine]
    sums, dg = D.metainfo_digest_host(datas, piece)  # the product path
    local = {i: (bytes(dg[k]).hex(), sums[k].tolist()) for k, i in enumerate(mine)}
    merged = gather_results(local, dist)
    if rank == 0:
        q.put(merged)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_product_path_gathered(orc):
    rng = np.random.default_rng(21)
    lens = rng.integers(0, 6 << 20, size=20)
    piece = 1 << 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lens, piece, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(merged) == list(range(len(lens)))
    shards = lpt_shard(lens, 2)
    assert shards[0] and shards[1]
    for i, L in enumerate(lens):
        data = orc.synth(i, int(L))
        assert merged[i][0] == hashlib.sha256(data.tobytes()).hexdigest()
        assert merged[i][1] == orc.calc_piece_sums(data, piece)[1].tolist()
