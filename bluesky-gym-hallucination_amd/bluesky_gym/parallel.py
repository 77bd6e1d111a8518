"""Multi-GPU: one process per GPU (torch.distributed over RCCL/xGMI), env shards with no
exchange during the step, and one all-gather per RL step of the learner rows
[obs..., reward, terminated, truncated] (fp32) so every rank sees the whole node's batch.

The gather of step t runs on a communication stream while step t+1's kernel runs on the
compute stream (double-buffered learner rows), so at 4096 envs per GPU the collective
hides behind the step.  Shards draw device spawns with global env ids (env_offset), so a
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


def all_gather_rows(out: torch.Tensor, local: torch.Tensor, group=None):
    """out[world*n, d] <- concat over ranks of local[n, d] (RCCL all_gather_into_tensor;
    list all_gather fallback for backends without it, e.g. some gloo builds)."""
    try:
        dist.all_gather_into_tensor(out, local, group=group)
    except (RuntimeError, AttributeError, NotImplementedError):
        world = dist.get_world_size(group)
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, local, group=group)
    return out


class ShardedVectorEnv:
    """Local shard of a node-wide vector env + per-step learner-row all-gather."""

    def __init__(self, make_local, total_envs: int, *, overlap=True, group=None):
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
        self.overlap = overlap and self.world > 1
        self._comm = torch.cuda.Stream(device=dev) if self.overlap else None
        self._done_ev = [None, None]

    def reset(self, **kw):
        return self.local.reset(**kw)

    def step(self, local_actions):
        """Steps the local shard; returns (gathered rows tensor, ready event).  The rows of
        this step are complete on every rank once `ready` has completed."""
        b = self.local.batch
        cur = self._cur
        if b.learner is not self._rows[cur]:
            b.learner = self._rows[cur]
            b._bind()
        self.local.step_tensors(local_actions)
        if self.world == 1:
            self._gathered[cur][: self.n_local].copy_(self._rows[cur])
            ev = torch.cuda.Event()
            ev.record()
        elif self.overlap:
            compute = torch.cuda.current_stream(b.device)
            ev_k = torch.cuda.Event()
            ev_k.record(compute)
            with torch.cuda.stream(self._comm):
                self._comm.wait_event(ev_k)
                all_gather_rows(self._gathered[cur], self._rows[cur], self.group)
                ev = torch.cuda.Event()
                ev.record(self._comm)
            # the kernel two steps ahead rewrites this buffer: make compute wait for the gather
            self._done_ev[cur] = ev
            nxt = 1 - cur
            if self._done_ev[nxt] is not None:
                compute.wait_event(self._done_ev[nxt])
        else:
            all_gather_rows(self._gathered[cur], self._rows[cur], self.group)
            ev = torch.cuda.Event()
            ev.record()
        self._cur = 1 - cur
        return self._gathered[cur], ev

    def close(self):
        self.local.close()
