"""Multi-GPU: one process per GPU (torch.distributed over RCCL/xGMI), env shards with no
exchange during the step, and an all-gather of the learner rows [obs..., reward,
terminated, truncated] (fp32) so every rank sees the whole node's batch -- one per RL step,
or one per block of k steps (steps_per_gather: fewer, larger collectives).

The gather of step t runs on RCCL's own stream while step t+1's kernel runs on the
compute stream (double-buffered learner rows, async Work handles), so at 4096 envs per
GPU the collective hides behind the step.  Shards draw device spawns with global env ids (env_offset), so a
sharded job is the same set of episodes as one big batch.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int):
    """Contiguous equal shards (all_gather_into_tensor needs equal sizes)."""
    if total % world:
        raise ValueError(f"total envs {total} must be divisible by world size {world}")
    n = total // world
    return rank * n, n


def all_gather_rows(out: torch.Tensor, local: torch.Tensor, group=None, async_op=False):
    """out[world*n, d] <- concat over ranks of local[n, d] (RCCL all_gather_into_tensor;
    list all_gather fallback for backends without it, e.g. some gloo builds).  With
    async_op the collective's Work handle is returned (else None after completion)."""
    try:
        return dist.all_gather_into_tensor(out, local, group=group, async_op=async_op)
    except (RuntimeError, AttributeError, NotImplementedError):
        world = dist.get_world_size(group)
        parts = list(out.chunk(world, dim=0))
        return dist.all_gather(parts, local, group=group, async_op=async_op)


class Ready:
    """Completion of one step's gathered rows.  wait(): the current stream (RCCL) or the
    host (gloo) waits until every rank's rows of that step are in the gathered buffer."""

    def __init__(self, work=None):
        self._work = work

    def wait(self):
        if self._work is not None:
            self._work.wait()


class ShardedVectorEnv:
    """Local shard of a node-wide vector env + the learner-row all-gather.

    Per step the host does: one bsg_step launch and one pointer swap of the learner rows
    (bsg_set_learner); per block of k = steps_per_gather steps one asynchronous
    all_gather_into_tensor of the block's k x [n_local, obs+3] rows.  RCCL runs it on its
    own stream after the block's last kernel, concurrently with the next block's kernels;
    the kernel that next rewrites the block's rows (two blocks later: the rows are a ring
    of two blocks) is ordered after it by Work.wait() (a stream wait, the host does not
    block).  The host side matters at C4's shard sizes: a 512-env shard's kernel is ~30 us,
    while one all_gather enqueue costs ~13-30 us and Work.wait ~7 us of host time
    (profiles/r03/shard_host_breakdown.txt) -- per step they made the loop host-bound;
    per block of 8 they are ~5 us a step.  (A full re-bind plus event bookkeeping per step
    cost ~70 us of host time, tools/shard_overhead.py.)

    k = 1 (default): step() returns (rows [total_envs, obs+3], Ready) every step.
    k > 1: step() returns (None, None) inside a block and, at the block's last step,
    (block, Ready) with block a [k, world, n_local, obs+3] view (step, rank, env of the
    rank; .reshape(k, total_envs, -1) gives global env order, as a copy).  flush()
    gathers a partial block (call it before reading the rows of the last steps)."""

    def __init__(self, make_local, total_envs: int, *, overlap=True, group=None, collective=None,
                 steps_per_gather: int = 1):
        """collective: optional ``f(out, rows) -> Work`` that starts the gather of this
        rank's rows into ``out`` asynchronously (``Work.wait()`` = a stream wait), in place
        of RCCL's all_gather_into_tensor -- another transport, or a test's delayed copy
        (tests/test_gpu_sharded.py).  With it the overlapped path is used at any world size."""
        if int(steps_per_gather) < 1:
            raise ValueError("steps_per_gather must be >= 1")
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.offset, self.n_local = shard_range(total_envs, self.world, self.rank)
        self.total_envs = total_envs
        self.k = int(steps_per_gather)
        self.local = make_local(num_envs=self.n_local, env_offset=self.offset, learner=True)
        b = self.local.batch
        d = b.obs_dim + 3
        self.row_dim = d
        dev = b.device
        # rows[blk, i]: the kernel's learner output of step i of block blk (a ring of 2 blocks)
        self._rows = torch.zeros((2, self.k, self.n_local, d), dtype=torch.float32, device=dev)
        self._gathered = [torch.empty((self.world * self.k, self.n_local, d), dtype=torch.float32,
                                      device=dev) for _ in range(2)]
        self._blk, self._i = 0, 0
        self._collective = collective
        self.overlap = collective is not None or (overlap and self.world > 1)
        self._work = [None, None]

    def _slot(self):
        """Point the kernel's learner output at the next slot; before the first write into a
        block, wait (on the stream) for that block's previous gather."""
        blk, i = self._blk, self._i
        if i == 0:
            w = self._work[blk]
            if w is not None:
                w.wait()
                self._work[blk] = None
        self.local.batch.set_learner(self._rows[blk, i])
        return blk, i

    def reset(self, **kw):
        """Resets the local shard and gathers every rank's reset rows (obs, reward 0,
        terminated 0, truncated 0) at once, as a block of one step: returns (rows, Ready)
        shaped as step() does (k = 1: [total_envs, obs+3]; k > 1: [1, world, n_local,
        obs+3]).  The local shard's Dict observation stays available as self.local_obs.
        k > 1: a block still open (steps taken since the last gather) raises -- call flush()
        first and keep its (block, Ready), or those steps' rows would never reach the caller."""
        if self._i:
            raise RuntimeError(f"reset() with {self._i} step(s) of an open gather block: "
                               "call flush() first and consume its rows")
        blk, _ = self._slot()
        # (a reset(seed=) that rebuilds the batch keeps the learner buffer: vector.py)
        self.local_obs, self.local_info = self.local.reset(**kw)
        return self._gather(blk, 1)

    def step(self, local_actions):
        """Steps the local shard.  k = 1: returns (gathered rows [total_envs, obs+3],
        Ready); they may be read after ready.wait(), until the step after next.  k > 1:
        (None, None) inside a block, (block, Ready) at its last step; a block stays valid
        until the end of the next block."""
        blk, i = self._slot()
        self.local.step_tensors(local_actions)
        if i + 1 < self.k:
            self._i = i + 1
            return None, None
        return self._gather(blk, self.k)

    def flush(self):
        """Gather the steps of the current partial block now (k > 1); (None, None) if the
        block is empty."""
        if self._i == 0:
            return None, None
        return self._gather(self._blk, self._i)

    def _gather(self, blk, n):
        src = self._rows[blk, :n]                       # [n, n_local, d], contiguous
        out = self._gathered[blk][: self.world * n]     # rank-major: out[r * n + i]
        if self.overlap:
            if self._collective is not None:
                work = self._collective(out, src)
            else:
                work = all_gather_rows(out, src, self.group, async_op=True)
            self._work[blk] = work
            ready = Ready(work)
        elif self.world == 1:
            out.copy_(src)
            ready = Ready()
        else:
            all_gather_rows(out, src, self.group)
            ready = Ready()
        self._blk, self._i = 1 - blk, 0
        if self.k == 1:
            return out.view(self.total_envs, self.row_dim), ready
        return out.view(self.world, n, self.n_local, self.row_dim).permute(1, 0, 2, 3), ready

    def close(self):
        for w in self._work:
            if w is not None:
                w.wait()
        self._work = [None, None]
        self.local.close()
