"""ShardedVectorEnv's block bookkeeping on the CPU (no GPU): world-size-2 gloo processes
drive it over a stand-in local env whose "kernel" writes known values into the learner
slot it is pointed at, so the test sees exactly which slot each step wrote and where the
gathered block puts it -- per step (k = 1) and per block (k = 3, with a partial block
flushed), overlapped and not.  The GPU tests (tests/test_gpu_sharded.py) check the same
path bit-exact against one device batch."""
import os
import socket

import pytest
import torch

D = 4                    # row width (obs 1 + reward, terminated, truncated)
N_LOCAL = 5
T = 10


class _Batch:
    def __init__(self, n):
        self.obs_dim = D - 3
        self.device = torch.device("cpu")
        self.learner = torch.zeros((n, D))
        self.n = n

    def set_learner(self, rows):
        assert rows.is_contiguous() and tuple(rows.shape) == (self.n, D)
        self.learner = rows


class _Local:
    """Writes value = 1000 * rank + 10 * step + column-independent env index into the
    learner rows (step -1 = reset)."""

    def __init__(self, num_envs, env_offset, learner):
        assert learner
        self.batch = _Batch(num_envs)
        self.rank = env_offset // num_envs
        self.t = -1

    def _write(self):
        env = torch.arange(self.batch.n, dtype=torch.float32)[:, None].expand(self.batch.n, D)
        self.batch.learner.copy_(1000.0 * self.rank + 10.0 * self.t + env)

    def reset(self, **kw):
        self.t = -1
        self._write()
        return {}, {}

    def step_tensors(self, actions):
        self.t += 1
        self._write()

    def close(self):
        pass


def _expected(world, t):
    env = torch.arange(N_LOCAL, dtype=torch.float32)
    return torch.cat([1000.0 * r + 10.0 * t + env for r in range(world)])   # [total]


def _worker(rank, world, port, k, overlap, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym.parallel import ShardedVectorEnv
        env = ShardedVectorEnv(_Local, world * N_LOCAL, overlap=overlap, steps_per_gather=k)
        got = {}

        def take(first_t, rows, ready):
            ready.wait()
            if rows.dim() == 2:
                got[first_t] = rows[:, 0].clone()
            else:
                for i in range(rows.shape[0]):
                    got[first_t + i] = rows[i].reshape(world * N_LOCAL, D)[:, 0].clone()

        rows, ready = env.reset()
        take(-1, rows, ready)
        block_start = 0
        for t in range(T):
            rows, ready = env.step(None)
            if rows is not None:
                take(block_start, rows, ready)
                block_start = t + 1
        rows, ready = env.flush()
        if rows is not None:
            take(block_start, rows, ready)
        env.close()
        q.put((rank, {t: v.tolist() for t, v in got.items()}, None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("k,overlap", [(1, True), (1, False), (3, True), (3, False), (8, True)])
def test_blocks_deliver_every_step_in_order(k, overlap):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got, err = q.get(timeout=120)
        assert err is None, f"rank {r}: {err}"
        res[r] = got
    for p in procs:
        p.join(timeout=30)
    for r in range(world):
        got = res[r]
        assert sorted(got) == list(range(-1, T)), sorted(got)     # reset + every step, once
        for t, v in got.items():
            assert v == _expected(world, t).tolist(), (r, t)


def _worker_midreset(rank, world, port, q):
    """k = 3: a reset() while a block is open must raise (it used to flush and
    drop the block's rows); after flush() the rows of the open block arrive and reset() works."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym.parallel import ShardedVectorEnv
        env = ShardedVectorEnv(_Local, world * N_LOCAL, overlap=True, steps_per_gather=3)
        env.reset()
        for _ in range(4):                       # one full block (t = 0..2), t = 3 opens one
            env.step(None)
        raised = False
        try:
            env.reset()
        except RuntimeError:
            raised = True
        rows, ready = env.flush()
        ready.wait()
        t3 = rows[0].reshape(world * N_LOCAL, D)[:, 0].tolist()
        rows, ready = env.reset()
        ready.wait()
        r = rows[0].reshape(world * N_LOCAL, D)[:, 0].tolist()
        env.close()
        q.put((rank, (raised, t3, r), None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_reset_with_an_open_block_raises_and_loses_nothing():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_midreset, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        r, got, err = q.get(timeout=120)
        assert err is None, f"rank {r}: {err}"
        raised, t3, rst = got
        assert raised
        assert t3 == _expected(world, 3).tolist()
        assert rst == _expected(world, -1).tolist()
    for p in procs:
        p.join(timeout=30)


def _worker_stale(rank, world, port, k, overlap, q):
    """A step's Ready stays valid for rows_valid_steps steps (its slot of the ring is not
    gathered into again before), its rows unchanged; after that wait() raises StaleRowsError
    (the views used to be overwritten silently)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym.parallel import ShardedVectorEnv, StaleRowsError
        env = ShardedVectorEnv(_Local, world * N_LOCAL, overlap=overlap, steps_per_gather=k)
        env.reset()
        held = None
        t = 0
        while held is None:                      # the first completed gather after the reset
            rows, ready = env.step(None)
            if rows is not None:
                held = (t - k + 1, rows, ready)
            t += 1
        t0, rows, ready = held
        ready.wait()
        first = rows.clone()
        n_ok = 0
        local_ok = []                             # local_rows(ready) still answers
        env.local_rows(ready)
        for _ in range(env.rows_valid_steps - 1):   # still inside the window
            env.step(None)
            try:
                env.local_rows(ready)
                local_ok.append(True)
            except StaleRowsError:
                local_ok.append(False)
            assert ready.valid
            ready.wait()
            assert torch.equal(rows, first)
            n_ok += 1
        for _ in range(k):                        # the step(s) that gather into its slot again
            env.step(None)
        raised = False
        try:
            ready.wait()
        except StaleRowsError:
            raised = True
        env.flush()
        env.close()
        q.put((rank, (env.rows_valid_steps, n_ok, raised, ready.valid, local_ok), None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,overlap", [(1, True), (1, False), (3, True)])
def test_stale_rows_raise(k, overlap):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_stale, args=(r, world, port, k, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        r, got, err = q.get(timeout=120)
        assert err is None, f"rank {r}: {err}"
        valid_steps, n_ok, raised, still_valid, local_ok = got
        assert valid_steps == 2 * k and n_ok == valid_steps - 1
        # this rank's own rows live until the kernel starts rewriting the slot: the first step
        # of the slot's next block (k > 1), k - 1 steps before the gathered rows go stale
        assert local_ok == [True] * k + [False] * (k - 1), local_ok
        assert raised and not still_valid
    for p in procs:
        p.join(timeout=30)


def _worker_rccl_fallback(rank, world, port, q):
    """RcclGather's construction is one decision for all ranks: with no usable
    device here every rank must raise BsgError -- none may be left blocked in a collective
    the others skipped -- and ShardedVectorEnv(transport='rccl') raises on both ranks alike."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bluesky_gym import _native as nat
        from bluesky_gym.parallel import RcclGather
        try:
            RcclGather(torch.device("cpu"))
            res = "constructed"
        except nat.BsgError as ex:
            res = "raised: " + str(ex)
        dist.barrier()                            # both ranks got here: nobody hangs
        q.put((rank, res, None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_rccl_transport_failure_is_collective():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_rccl_fallback, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, res, err = q.get(timeout=120)
        assert err is None, f"rank {r}: {err}"
        got[r] = res
    for p in procs:
        p.join(timeout=30)
    assert all(v.startswith("raised") for v in got.values()), got
