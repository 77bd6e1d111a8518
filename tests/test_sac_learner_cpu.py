"""The SAC learner of bench.py --workload descent-sac (tools/sac_torch.py) on the CPU:
the reference's saved actor loads into it and reproduces tests/ref_policy.py's actor,
the replay ring buffer wraps, updates run and change the networks, and the
data-parallel gradient all-reduce of two gloo ranks equals one learner on the union
batch (world-size-2 rehearsal of the multi-GPU learner)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import sac_torch  # noqa: E402
import ref_policy as sp  # noqa: E402


def test_actor_loads_reference_weights():
    W = sp.load()
    a = sac_torch.Actor(4, 1)
    a.load_sb3(W, "descent")
    obs = np.random.default_rng(0).standard_normal((64, 4)).astype(np.float32)
    h = a.latent(torch.from_numpy(obs))
    mu = a.mu(h).detach().numpy()
    np.testing.assert_allclose(np.tanh(mu), sp.actor_np(W, "descent", obs), rtol=1e-5, atol=1e-6)


def test_buffer_and_updates():
    torch.manual_seed(0)
    s = sac_torch.SAC(4, 1, "cpu", buffer=100, batch=16)
    for k in range(30):
        o = torch.randn(8, 4)
        a = torch.rand(8, 1) * 2 - 1
        s.insert(o, a, torch.randn(8), torch.randn(8, 4), (torch.rand(8) < 0.1).float())
    assert int(s.size) == 100 and int(s.pos) == (30 * 8) % 100
    before = [p.detach().clone() for p in s.q1.parameters()]
    for _ in range(5):
        lq, la = s.update()
        assert torch.isfinite(lq) and torch.isfinite(la)
    assert any(not torch.equal(b, p) for b, p in zip(before, s.q1.parameters()))


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = sac_torch.SAC(4, 1, "cpu", buffer=64, batch=32, group=dist.group.WORLD, seed=0)
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(16, 4, generator=g)
        s.insert(x, torch.zeros(16, 1), torch.ones(16), x, torch.zeros(16))
        o, a, r, o2, d = s.buf_obs[:16], s.buf_act[:16], s.buf_rew[:16], s.buf_next[:16], s.buf_done[:16]
        xin = torch.cat([o, a], -1)
        loss = s.q1(xin).pow(2).mean()
        s.opt_q.zero_grad(set_to_none=False)
        loss.backward()
        s._allreduce(list(s.q1.parameters()))
        q.put((rank, [p.grad.numpy().copy() for p in s.q1.parameters()], x.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gradient_allreduce_equals_union_batch():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, x)) for r, g, x in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
    # same init on both ranks (seed 0): one learner on both ranks' samples
    s = sac_torch.SAC(4, 1, "cpu", buffer=64, batch=32, seed=0)
    xs = torch.from_numpy(np.concatenate([res[0][1], res[1][1]]))
    loss = s.q1(torch.cat([xs, torch.zeros(32, 1)], -1)).pow(2).mean()
    loss.backward()
    for g0, g1, p in zip(res[0][0], res[1][0], s.q1.parameters()):
        np.testing.assert_array_equal(g0, g1)
        np.testing.assert_allclose(g0, p.grad.numpy(), rtol=1e-5, atol=1e-6)


def _dp_seed_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # bench.py's construction: the rank is the sampling seed
        s = sac_torch.SAC(4, 1, "cpu", buffer=64, batch=32, group=dist.group.WORLD, seed=rank)
        g = torch.Generator().manual_seed(100 + rank)
        for _ in range(4):
            x = torch.randn(16, 4, generator=g)
            s.insert(x, torch.rand(16, 1, generator=g) * 2 - 1, torch.randn(16, generator=g),
                     torch.randn(16, 4, generator=g), torch.zeros(16))
        for _ in range(3):
            lq, la = s.update()
            assert torch.isfinite(lq) and torch.isfinite(la)
        nets = (list(s.actor.parameters()) + list(s.q.parameters()) + list(s.qt.parameters())
                + [s.log_alpha])
        q.put((rank, [p.detach().numpy().copy() for p in nets]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_different_seeds_same_parameters():
    """each rank seeds SAC with its own rank (its replay draws and noise), yet
    the ranks are one data-parallel learner -- rank 0's networks are broadcast at
    construction and the mean gradient keeps them equal, update after update."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_seed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)
