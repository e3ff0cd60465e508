"""The multi-GPU plumbing on CPU (gloo, world size 2): request sharding, the out-of-band RCCL id
exchange, and that every rank compiles the identical image (so an RCCL-broadcast image and a
locally compiled one are interchangeable). The RCCL broadcast itself needs GPUs (test_gpu_parity)."""
import hashlib
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import cedargpu
from cedargpu import dist as cdist
from cedargpu import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_covers_disjointly():
    for n in (0, 1, 7, 65536, 100003):
        for world in (1, 2, 3, 8):
            ranges = [cdist.shard(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        cdist.shard(10, 2, 2)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        uid = cdist.exchange_unique_id(rank, make=lambda: bytes(range(128)))
        pop = synth.Population(seed=3, n_users=200, n_groups=20)
        image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(300, seed=3, pop=pop))], epoch=7)
        digest = hashlib.sha256(image).hexdigest()
        got = [None] * world
        dist.all_gather_object(got, (digest, uid, cdist.shard(1000, rank, world)))
        if rank == 0:
            out.put(got)
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == got[1][0]                      # identical compiled image on both ranks
    assert got[0][1] == got[1][1] == bytes(range(128))  # the id reached rank 1
    assert got[0][2] == (0, 500) and got[1][2] == (500, 1000)
