"""Multi-GPU: one process per GPU (torch.distributed over RCCL/xGMI), env shards with no
exchange during the step, and one all-gather per RL step of the learner rows
[obs..., reward, terminated, truncated] (fp32) so every rank sees the whole node's batch.

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
    """Local shard of a node-wide vector env + per-step learner-row all-gather.

    Per step the host does: one bsg_step launch, one pointer swap of the learner rows
    (bsg_set_learner) and one asynchronous all_gather_into_tensor -- RCCL runs it on its
    own stream after the step kernel, concurrently with the next step's kernel; the
    kernel two steps later, which rewrites the same rows buffer, is ordered after it by
    Work.wait() (a stream wait, the host does not block).  Keeping the host side to these
    three calls matters: a full re-bind plus event bookkeeping per step cost ~70 us of host
    time, as much as the kernel itself (tools/shard_overhead.py)."""

    def __init__(self, make_local, total_envs: int, *, overlap=True, group=None, collective=None):
        """collective: optional ``f(out, rows) -> Work`` that starts the gather of this
        rank's rows into ``out`` asynchronously (``Work.wait()`` = a stream wait), in place
        of RCCL's all_gather_into_tensor -- another transport, or a test's delayed copy
        (tests/test_gpu_sharded.py).  With it the overlapped path is used at any world size."""
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.offset, self.n_local = shard_range(total_envs, self.world, self.rank)
        self.local = make_local(num_envs=self.n_local, env_offset=self.offset, learner=True)
        b = self.local.batch
        d = b.obs_dim + 3
        dev = b.device
        self._rows = [b.learner, torch.zeros_like(b.learner)]
        self._gathered = [torch.empty((total_envs, d), dtype=torch.float32, device=dev)
                          for _ in range(2)]
        self._cur = 0
        self._collective = collective
        self.overlap = collective is not None or (overlap and self.world > 1)
        self._work = [None, None]

    def _swap_in(self):
        """rows[cur] becomes the kernel's learner output, once the gather two launches ago
        (which reads the same buffer) is done."""
        b = self.local.batch
        cur = self._cur
        w = self._work[cur]
        if w is not None:
            w.wait()
            self._work[cur] = None
        if b.learner is not self._rows[cur]:
            b.set_learner(self._rows[cur])
        return cur

    def reset(self, **kw):
        """Resets the local shard and gathers every rank's reset rows (obs, reward 0,
        terminated 0, truncated 0): returns (gathered rows [total_envs, obs+3], Ready) like
        step(), so a learner on any rank sees the node's first observations.  The local
        shard's Dict observation stays available as self.local_obs."""
        cur = self._swap_in()
        # (a reset(seed=) that rebuilds the batch keeps the learner buffer: vector.py)
        self.local_obs, self.local_info = self.local.reset(**kw)
        assert self.local.batch.learner is self._rows[cur]
        return self._gather(cur)

    def step(self, local_actions):
        """Steps the local shard; returns (gathered rows [total_envs, obs+3], Ready).  The
        rows of this step may be read after ready.wait(), until the step after next."""
        cur = self._swap_in()
        self.local.step_tensors(local_actions)
        return self._gather(cur)

    def _gather(self, cur):
        if self.overlap:
            if self._collective is not None:
                work = self._collective(self._gathered[cur], self._rows[cur])
            else:
                work = all_gather_rows(self._gathered[cur], self._rows[cur], self.group,
                                       async_op=True)
            self._work[cur] = work
            ready = Ready(work)
        elif self.world == 1:
            self._gathered[cur][: self.n_local].copy_(self._rows[cur])
            ready = Ready()
        else:
            all_gather_rows(self._gathered[cur], self._rows[cur], self.group)
            ready = Ready()
        self._cur = 1 - cur
        return self._gathered[cur], ready

    def close(self):
        for w in self._work:
            if w is not None:
                w.wait()
        self._work = [None, None]
        self.local.close()
