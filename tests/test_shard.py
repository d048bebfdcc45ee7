"""Multi-GPU path on CPU: the batch sharding and the per-step publish
all-gather of bench.py (openkite_amd/shard.py), world_size 2 over gloo."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openkite_amd.shard import PUB_COLS, Publisher, max_over_ranks, shard


def test_shard_partitions_batch():
    for G in (1, 2, 3, 8):
        for B in (1, 7, 4096, 32768):
            parts = [shard(B, G, r) for r in range(G)]
            assert sum(c for _, c in parts) == B
            off = 0
            for o, c in parts:
                assert o == off and abs(c - B // G) <= 1
                off += c


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt = shard(world * B, world, rank)
        assert cnt == B
        ids = torch.arange(off, off + cnt, dtype=torch.float64)
        u0 = ids[:, None] * 10 + torch.arange(4, dtype=torch.float64)
        diag = -ids[:, None] * 10 - torch.arange(6, dtype=torch.float64)
        pub = Publisher(B, "cpu", world)
        g = pub.publish(u0, diag)
        t = max_over_ranks(0.5 + rank, "cpu")
        q.put((rank, g.clone(), t))
    finally:
        dist.destroy_process_group()


def test_publish_allgather_world2_gloo():
    world, B = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ids = torch.arange(world * B, dtype=torch.float64)
    want = torch.cat([ids[:, None] * 10 + torch.arange(4, dtype=torch.float64),
                      -ids[:, None] * 10 - torch.arange(6, dtype=torch.float64)], dim=1)
    for rank, g, t in res:
        assert g.shape == (world * B, PUB_COLS)
        assert torch.equal(g, want), rank          # rank order, every rank sees every kite
        assert t == 0.5 + (world - 1)              # slowest rank's time
