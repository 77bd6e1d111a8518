"""The multi-GPU code path on the one-GPU box: ShardedVectorEnv with 2 ranks (gloo, both
on cuda:0) against one un-sharded DeviceBatch of all the envs -- the gathered
[E, obs+3] learner rows must be bit-identical every step, through reset and autoresets,
with the asynchronous gather overlapped (Work handles, double-buffered rows, the
pointer swap two steps later).  Replaces the reference's SubprocVecEnv
(scripts/multi_processing_example.py:51-53).  Also: the Gymnasium reset-seeding
contract, the SAME_STEP/host-spawn guard and the SectorCR capacity flag."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

E_LOCAL, T, SEED, MAXEP = 128, 64, 77, 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _actions(total):
    g = torch.Generator().manual_seed(5)
    return torch.rand((T, total, 2), dtype=torch.float64, generator=g) * 2 - 1


def _rows_list(rows, total):
    """The per-step [total, d] rows of a gathered result (k = 1: one step; k > 1: a block
    [n, world, n_local, d])."""
    if rows.dim() == 2:
        return [rows.cpu().numpy().copy()]
    return [rows[i].reshape(total, -1).cpu().numpy().copy() for i in range(rows.shape[0])]


def _shard_worker(rank, world, port, overlap, k, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym.parallel import ShardedVectorEnv
        from bluesky_gym.vector import MergeVectorEnv
        total = world * E_LOCAL
        env = ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=SEED, compute_cd=True,
                                                           max_episode_steps=MAXEP, **kw),
                               total, overlap=overlap, steps_per_gather=k)
        acts = _actions(total)
        rows, ready = env.reset()
        ready.wait()
        torch.cuda.synchronize()
        out = _rows_list(rows, total)
        for t in range(T):
            a = acts[t, env.offset:env.offset + env.n_local].cuda()
            rows, ready = env.step(a)
            if rows is None:
                continue
            ready.wait()
            torch.cuda.synchronize()
            out += _rows_list(rows, total)
        env.close()
        q.put((rank, np.stack(out) if rank == 0 else None, None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap,k", [(True, 1), (False, 1), (True, 4), (True, 8)])
def test_sharded_rows_match_one_batch(overlap, k):
    """k = steps_per_gather: one all-gather per step, or per block of 4 steps."""
    import torch.multiprocessing as mp
    from bluesky_gym import config, core
    world = 2
    total = world * E_LOCAL
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, overlap, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, arr, err = q.get(timeout=240)
        assert err is None, f"rank {r}: {err}"
        res[r] = arr
    for p in procs:
        p.join(timeout=60)
    got = res[0]
    # the same envs as one batch (global env ids 0..total-1 -> same Philox spawns)
    b = core.DeviceBatch(config.merge_config(num_ac=32, max_episode_steps=MAXEP), total,
                         compute_cd=True, seed=SEED, learner=True)
    acts = _actions(total)
    b.reset()
    torch.cuda.synchronize()
    want = [b.learner.cpu().numpy().copy()]
    done = 0
    for t in range(T):
        b.step(acts[t].cuda())
        want.append(b.learner.cpu().numpy().copy())
        done += int((b.terminated | b.truncated).sum())
    want = np.stack(want)
    assert done >= total * (T // MAXEP), done        # autoresets happened in the window
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
        np.argwhere(got.view(np.uint32) != want.view(np.uint32))[:5]


class _DelayedGather:
    """A stand-in for RCCL's asynchronous all_gather_into_tensor with RCCL's stream
    semantics: the collective's stream waits for the caller's stream at enqueue, then (here)
    spins for a long delay before it reads the rows; Work.wait() makes the caller's
    current stream wait for the copy's completion event (the host never blocks).
    honour_wait=False is the negative control, made deterministic: a collective that reads
    its rows only when the NEXT collective is enqueued -- after the kernels in between, so
    whatever they rewrote is what it gathers -- with a wait() that orders nothing.  (A
    delayed copy alone is not a reliable control: when the side stream shares a hardware
    queue with the compute stream the two serialise and the hazard never shows.)"""

    def __init__(self, delay_cycles, honour_wait=True):
        self.side = torch.cuda.Stream()
        self.delay = delay_cycles
        self.honour = honour_wait
        self.pending = None

    def __call__(self, out, rows):
        cur = torch.cuda.current_stream()
        if not self.honour:
            if self.pending is not None:
                po, pr = self.pending
                po[: pr.shape[0]].copy_(pr)          # on the compute stream, one call late
            self.pending = (out, rows)

            class NoWork:
                def wait(self):
                    pass
            return NoWork()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            torch.cuda._sleep(self.delay)
            out[: rows.shape[0]].copy_(rows)
            done = torch.cuda.Event()
            done.record(self.side)

        class Work:
            def wait(self):
                torch.cuda.current_stream().wait_event(done)
        return Work()


def _ordering_run(gather, T_steps=64, E=256, k=1):
    """ShardedVectorEnv (one rank) over the delayed gather, with no host sync between steps:
    each gathered step's rows are cloned on the compute stream after ready.wait()."""
    from bluesky_gym.parallel import ShardedVectorEnv
    from bluesky_gym.vector import MergeVectorEnv
    env = ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=SEED, compute_cd=True,
                                                       max_episode_steps=MAXEP, **kw),
                           E, collective=gather, steps_per_gather=k)
    g = torch.Generator().manual_seed(9)
    acts = (torch.rand((T_steps, E, 2), dtype=torch.float64, generator=g) * 2 - 1).cuda()
    hist = []
    def take(rows):
        return [rows.clone()] if rows.dim() == 2 else [rows[i].reshape(E, -1).clone()
                                                        for i in range(rows.shape[0])]
    rows, ready = env.reset()
    ready.wait()
    hist += take(rows)
    for t in range(T_steps):
        rows, ready = env.step(acts[t])
        if rows is None:
            continue
        ready.wait()
        hist += take(rows)
    torch.cuda.synchronize()
    env.close()
    return torch.stack(hist).cpu().numpy(), acts


@pytest.mark.parametrize("k", [1, 4])
def test_overlapped_gather_never_reads_rewritten_rows(k):
    """the stream ordering of ShardedVectorEnv's overlapped gather.  The
    kernel that next writes a block's rows (two blocks later: k = 1, the step after next)
    rewrites the buffer that block's gather reads; _slot's Work.wait() must order it after
    that (delayed) read.  Bit-exact against one batch over 64 steps with autoresets; the
    negative control (a wait() that orders nothing) must be caught by the same comparison,
    so the test can see the hazard it guards against.  k = 4: blocks of 4 steps per gather."""
    from bluesky_gym import config, core
    delay = 1_000_000                   # >> one 256-env step kernel at either clock rate
    got, acts = _ordering_run(_DelayedGather(delay), k=k)
    E = acts.shape[1]
    b = core.DeviceBatch(config.merge_config(num_ac=32, max_episode_steps=MAXEP), E,
                         compute_cd=True, seed=SEED, learner=True)
    b.reset()
    want = [b.learner.clone()]
    for t in range(acts.shape[0]):
        b.step(acts[t])
        want.append(b.learner.clone())
    want = torch.stack(want).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
        np.argwhere(got.view(np.uint32) != want.view(np.uint32))[:5]
    bad, _ = _ordering_run(_DelayedGather(delay, honour_wait=False), k=k)
    assert not np.array_equal(bad.view(np.uint32), want.view(np.uint32)), \
        "the un-ordered control gathered correct rows: the delay does not expose the hazard"


def test_reset_with_seed_is_reproducible():
    from bluesky_gym.vector import MergeVectorEnv
    env = MergeVectorEnv(num_envs=64, num_ac=16, seed=0)
    o1, _ = env.reset(seed=3)
    a = np.random.default_rng(0).uniform(-1, 1, (64, 2))
    s1 = env.step(a)[0]
    o2, _ = env.reset(seed=3)
    s2 = env.step(a)[0]
    for k in o1:
        assert np.array_equal(o1[k], o2[k]), k
        assert np.array_equal(s1[k], s2[k]), k
    o3, _ = env.reset()                       # no seed: the episode streams continue
    assert any(not np.array_equal(o1[k], o3[k]) for k in o1)
    env.close()


def test_sector_capacity_overflow_raises():
    """SectorCR draws 5..~40 aircraft per episode (sector_cr_env.py:95-100); with capacity
    num_ac=8 most episodes overflow: the device flags them and the env raises, as the
    host-spawn path does."""
    from bluesky_gym.vector import SectorCRVectorEnv
    env = SectorCRVectorEnv(num_envs=64, num_ac=8, seed=1)
    with pytest.raises(RuntimeError, match="more aircraft"):
        env.reset()
    env.close()
    ok = SectorCRVectorEnv(num_envs=64, num_ac=64, seed=1)   # capacity 64: P(overflow) ~ 0
    ok.reset()
    for _ in range(3):
        ok.step(np.zeros((64, 2)))
    ok.close()


def test_sector_overflow_check_is_lazy_on_the_tensor_path():
    """step_tensors() adds no host sync per call: the overflow flag is OR-ed on the device
    and read back every OVERFLOW_CHECK_EVERY calls, so an overflowing batch
    raises at that call and not before."""
    import torch
    from bluesky_gym.vector import SectorCRVectorEnv
    env = SectorCRVectorEnv(num_envs=64, num_ac=8, seed=1)
    with pytest.raises(RuntimeError, match="more aircraft"):
        env.reset()                                  # the flag persists until the next reset
    K = env.OVERFLOW_CHECK_EVERY
    a = torch.zeros((64, 2), dtype=torch.float64, device=env.batch.device)
    for _ in range(K - 1):
        env.step_tensors(a)
    with pytest.raises(RuntimeError, match="more aircraft"):
        env.step_tensors(a)
    env.close()


def test_sector_overflow_noted_by_step_tensors_is_raised_at_close():
    """fewer than OVERFLOW_CHECK_EVERY step_tensors() calls after an overflowing
    reset must still raise -- at close() (or the next reset()) -- never be lost."""
    import torch
    from bluesky_gym.vector import SectorCRVectorEnv
    env = SectorCRVectorEnv(num_envs=64, num_ac=8, seed=1)
    with pytest.raises(RuntimeError, match="more aircraft"):
        env.reset()
    a = torch.zeros((64, 2), dtype=torch.float64, device=env.batch.device)
    for _ in range(3):
        env.step_tensors(a)                      # the persisting flag is noted, not raised
    with pytest.raises(RuntimeError, match="more aircraft"):
        env.close()


@pytest.mark.parametrize("k", [1, 4, 8])
def test_rccl_transport_rows_match_one_batch(k):
    """The native RCCL gather (parallel.RcclGather: libbsg's bsg_comm_* -- ncclAllGather on
    a comm-owned stream, events per slot) on a one-rank communicator: the gathered rows are
    the un-sharded batch's, bit for bit, every step through autoresets, with the gather
    overlapped and the row ring reused (k = 1: every step; k = 4: per block).  RCCL cannot
    run two ranks on one GPU; the rank-major layout is the same call torch's
    all_gather_into_tensor makes (the 2-rank tests above)."""
    import torch.distributed as dist
    from bluesky_gym import config, core
    from bluesky_gym.parallel import ShardedVectorEnv
    from bluesky_gym.vector import MergeVectorEnv
    assert not dist.is_initialized()
    total = E_LOCAL
    env = ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=SEED, compute_cd=True,
                                                       max_episode_steps=MAXEP, **kw),
                           total, steps_per_gather=k, transport="rccl")
    assert env.transport == "rccl" and env.overlap
    info = env._rccl.info()                     # RCCL's own view (ncclCommCount / UserRank)
    assert info["nranks"] == 1 and info["rank"] == 0 and info["gathers"] == 0
    acts = _actions(total)
    got = []
    rows, ready = env.reset()
    ready.wait()
    got += _rows_list(rows, total)
    for t in range(T):
        rows, ready = env.step(acts[t].cuda())
        if rows is None:
            continue
        ready.wait()
        got += _rows_list(rows, total)    # (.cpu() on the current stream: after the wait)
    rows, ready = env.flush()
    if rows is not None:
        ready.wait()
        got += _rows_list(rows, total)
    assert env._rccl.info()["gathers"] == 1 + -(-T // k)     # the reset's + one per block
    env.close()
    b = core.DeviceBatch(config.merge_config(num_ac=32, max_episode_steps=MAXEP), total,
                         compute_cd=True, seed=SEED, learner=True)
    b.reset()
    want = [b.learner.cpu().numpy().copy()]
    for t in range(T):
        b.step(acts[t].cuda())
        want.append(b.learner.cpu().numpy().copy())
    got, want = np.stack(got), np.stack(want)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_rccl_graph_cache_serves_the_ring(monkeypatch):
    """BSG_COMM_GRAPHS=1 (the gather as a replayed HIP graph): the cache holds one graph per
    slot of the fused per-step path's ring, so after one lap every gather is a replay
    (an 8-entry FIFO missed on every one of the 16 slots).  Rows bit-identical to
    the plain ncclAllGather path."""
    from bluesky_gym.parallel import ShardedVectorEnv
    from bluesky_gym.vector import MergeVectorEnv
    from bluesky_gym import _native as nat
    total = E_LOCAL
    acts = _actions(total)
    out = {}
    for graphs in ("0", "1"):
        monkeypatch.setenv("BSG_COMM_GRAPHS", graphs)
        env = ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=SEED, compute_cd=True,
                                                           max_episode_steps=MAXEP, **kw),
                               total, steps_per_gather=1, transport="rccl")
        assert env._fused
        env.reset()[1].wait()
        got = []
        for t in range(T):
            rows, ready = env.step(acts[t].cuda())
            ready.wait()
            got.append(rows.cpu().numpy().copy())
        info = env._rccl.info()
        env.close()
        out[graphs] = (np.stack(got), info)
    info = out["1"][1]
    assert info["use_graphs"] == 1 and info["gathers"] == T + 1
    # the reset's gather (slot 0, a [1, n, d] block) and one capture per slot of the ring
    assert info["graph_captures"] <= nat.COMM_SLOTS + 1
    assert info["graph_hits"] == info["gathers"] - info["graph_captures"] and info["graph_hits"] > 0
    assert np.array_equal(out["0"][0].view(np.uint32), out["1"][0].view(np.uint32))
