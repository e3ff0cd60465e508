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


# ------------------------------------------------ multi-context queue + reload (device stand-in)
STUB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "san", "libcedargpu_stub.so")


def _queue_worker(rank, world, port, out):
    """One rank = one process with two contexts (GPUs) behind one serving queue. Rank 0 compiles,
    the blob travels over the collective (gloo here, RCCL on GPUs), every rank loads it on its first
    context and peer-copies it to the second; a reload then happens while callers keep calling."""
    import threading

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cedargpu as cg
        assert cg._lib.SANITIZER_BUILD  # the host engine over the device stand-in
        pop = synth.Population(seed=3, n_users=200, n_groups=20)
        text = synth.abac_policies(300, seed=3, pop=pop)

        comp = cg.Compiler() if rank == 0 else None
        prev = {}

        def reload(epoch, extra="", delta=False):
            # the second reload travels as a delta image against the first (cg_image_load_delta)
            blob = comp.build([cg.MemoryStore("c3.cedar", text + extra)], epoch=epoch) if rank == 0 else None
            msg = [cg.image_delta(prev["blob"], blob) if (rank == 0 and delta) else blob]
            if rank == 0:
                prev["blob"] = blob
            dist.broadcast_object_list(msg, src=0)
            if delta:
                ctxs[0].load_delta(epoch - 1, msg[0], epoch)
            else:
                ctxs[0].load(msg[0], epoch)    # new requests encode against it from here on
            ctxs[1].load_peer(ctxs[0], epoch)  # the second GPU follows (its batches fall back meanwhile)

        ctxs = [cg.Context(2 * rank), cg.Context(2 * rank + 1)]
        reload(1)
        q = cg.Queue(ctxs, max_batch=64, max_delay_us=50)
        sars = synth.random_sars(2000, seed=40 + rank, pop=pop)
        errors = []

        def caller(k):
            for s in sars[k::8]:
                try:
                    d, _ = q.authorize(s)
                    assert d in (0, 1, 2)
                except Exception as e:  # noqa: BLE001 (reported to the parent)
                    errors.append(repr(e))

        th = [threading.Thread(target=caller, args=(k,)) for k in range(8)]
        for t in th:
            t.start()
        reload(2, '\nforbid (principal, action == k8s::Action::"reload-check", resource);', delta=True)
        for t in th:
            t.join()
        stats = q.gpu_stats()
        q.close()
        if comp:
            comp.close()
        active = []
        for c in ctxs:
            e = cg._lib.u64()
            cg.lib.cg_image_active(c._h, cg._lib.ctypes.byref(e))
            active.append(e.value)
            c.close()
        got = [None] * world
        dist.all_gather_object(got, (errors, stats, active))
        if rank == 0:
            out.put(got)
    finally:
        dist.destroy_process_group()


def test_two_ranks_multi_context_queue_with_reload():
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # a fresh checkout has no build/san yet: name csrc from the repo root, not through build/san/..
    subprocess.run(["make", "-s", "-C", os.path.join(root, "cedar-access-control-for-k8s_amd", "csrc"), "stub"],
                   check=True, capture_output=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    old = os.environ.get("CEDARGPU_SANITIZER_LIB")
    os.environ["CEDARGPU_SANITIZER_LIB"] = STUB  # inherited by the spawned ranks only
    try:
        procs = [ctx.Process(target=_queue_worker, args=(r, 2, port, q)) for r in range(2)]
        for p in procs:
            p.start()
    finally:
        if old is None:
            del os.environ["CEDARGPU_SANITIZER_LIB"]
        else:
            os.environ["CEDARGPU_SANITIZER_LIB"] = old
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for errors, stats, active in got:
        assert errors == []
        assert sum(s["requests"] for s in stats) > 0
        assert all(s["batches"] > 0 for s in stats), stats  # both contexts of the rank ran batches
        assert active == [2, 2]                               # the reload reached both contexts
