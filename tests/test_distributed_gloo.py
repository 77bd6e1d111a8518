"""Multi-process (world_size 2, gloo, CPU) checks of the multi-GPU sharding and the
learner-row all-gather (bluesky_gym/parallel.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bluesky_gym.parallel import all_gather_rows, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total, d = 8, 43
        off, n = shard_range(total, world, rank)
        local = torch.arange(off * d, (off + n) * d, dtype=torch.float32).reshape(n, d)
        out = torch.empty((total, d), dtype=torch.float32)
        all_gather_rows(out, local)
        ok = torch.equal(out, torch.arange(total * d, dtype=torch.float32).reshape(total, d))
        q.put((rank, off, n, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_shard_range():
    assert [shard_range(4096, 8, r) for r in (0, 7)] == [(0, 512), (3584, 512)]
    with pytest.raises(ValueError):
        shard_range(10, 4, 0)


def test_gloo_world2_gather_rows():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, 0, 4, True), (1, 4, 4, True)]


def _async_worker(rank, world, port, q):
    """all_gather_rows(async_op=True) returns a Work handle whose wait() completes the
    gather (the ShardedVectorEnv overlap path); gloo on CPU."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym.parallel import Ready
        total, d = 6, 5
        off, n = shard_range(total, world, rank)
        local = torch.full((n, d), float(rank + 1))
        out = torch.zeros((total, d))
        work = all_gather_rows(out, local, async_op=True)
        Ready(work).wait()
        ok = bool(torch.equal(out[:3], torch.ones(3, d)) and torch.equal(out[3:], 2 * torch.ones(3, d)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_async_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, True), (1, True)]
