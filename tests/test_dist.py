"""CPU multi-process test of the sharding / key-broadcast layer (gloo, world_size 2)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from exacto_amd.dist import broadcast_key, gather_to, max_over_ranks, shard


def test_shard_covers_exactly():
    for total in (0, 1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard(total, r, world)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # key made on rank 0 only, identical everywhere after the broadcast
        key = torch.arange(2 * 3 * 16, dtype=torch.int64).reshape(1, 2, 3, 16) if rank == 0 else \
            torch.zeros((1, 2, 3, 16), dtype=torch.int64)
        broadcast_key(key)
        ok_key = bool(torch.equal(key, torch.arange(96, dtype=torch.int64).reshape(1, 2, 3, 16)))
        # each rank "computes" its shard; the gather reassembles the global batch in order
        total = 5
        s, c = shard(total, rank, world)
        out = torch.arange(s, s + c, dtype=torch.int64).reshape(c, 1) * 10
        full = gather_to(out, total)
        ok_gather = True if rank != 0 else bool(torch.equal(full.flatten(), torch.arange(total) * 10))
        t = max_over_ranks(float(rank + 1))
        q.put((rank, ok_key, ok_gather, t))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_shard_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok_key, ok_gather, t in res:
        assert ok_key and ok_gather and t == 2.0
