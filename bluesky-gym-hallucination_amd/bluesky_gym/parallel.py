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


class RcclGather:
    """The learner-row all-gather as direct RCCL calls from libbsg (include/bsg.h bsg_comm_*):
    per gather one C call -- an event on the caller's stream, ncclAllGather on the comm's own
    stream, a completion event per slot -- instead of torch.distributed's c10d enqueue
    (~28 us of host time per call, plus ~7 us per Work.wait: profiles/r03/
    shard_host_breakdown_k1.txt), which made a per-step gather the loop's bottleneck at
    C4's shard sizes.  The communicator's id is broadcast once over the process group."""

    def __init__(self, device, group=None):
        """Collective: every rank of `group` must construct it.  The transport is decided for
        all ranks at once: rank 0 broadcasts its id draw's status with the id, and
        after bsg_comm_create the ranks agree (an all-reduce of a success flag, RCCL's own
        rank count and rank included) before any gather -- so either every rank holds a
        communicator of `world` ranks, or every rank raises BsgError and the caller can fall
        back on all ranks together.  (A failure inside ncclCommInitRank that leaves the other
        ranks blocked in it cannot be caught here: RCCL's init is itself collective.)"""
        import ctypes as C
        from . import _native as nat
        self._C, self._nat = C, nat
        self.lib = nat.load_library()
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self._comm = C.c_void_p()
        self._dev = torch.device(device).index or 0
        on_dev = self.world > 1 and dist.get_backend(group) == "nccl"
        src = dist.get_global_rank(group, 0) if group is not None else 0
        # byte 0: rank 0's status (1 = the id was drawn), then the id
        idb = torch.zeros(1 + nat.COMM_ID_BYTES, dtype=torch.uint8)
        err = ""
        if self.rank == 0:
            rc = self.lib.bsg_comm_unique_id(C.c_void_p(idb.data_ptr() + 1))
            if rc == 0:
                idb[0] = 1
            else:
                err = self.lib.bsg_comm_last_error().decode(errors="replace")
        if self.world > 1:
            # the process group's backend decides where the id travels (RCCL: a device tensor)
            t = idb.to(device) if on_dev else idb
            dist.broadcast(t, src=src, group=group)
            idb = t.cpu()
        if int(idb[0]) != 1:
            raise nat.BsgError("RcclGather: rank 0 could not draw the RCCL id"
                               + (f": {err}" if err else " (see rank 0's error)"))
        comm = C.c_void_p()
        rc = self.lib.bsg_comm_create(C.c_void_p(idb.data_ptr() + 1), self.world, self.rank,
                                      self._dev, C.byref(comm))
        ok = rc == 0
        err = "" if ok else self.lib.bsg_comm_last_error().decode(errors="replace")
        if ok:
            self._comm = comm
            # (a failing info() must not keep this rank from the flag all-reduce below, where
            # the other ranks wait: ADVICE r05)
            try:
                info = self.info()
            except nat.BsgError as ex:
                ok, err = False, str(ex)
            else:
                if info["nranks"] != self.world or info["rank"] != self.rank:
                    ok = False
                    err = (f"RCCL sees {info['nranks']} ranks with this one as rank {info['rank']}, "
                           f"the process group {self.world} / {self.rank}")
        if self.world > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            flag = flag.to(device) if on_dev else flag
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            all_ok = int(flag.item()) == 1
        else:
            all_ok = ok
        if not all_ok:
            self.close()
            raise nat.BsgError("RcclGather: the communicator could not be created on every rank"
                               + (f"; this rank: {err}" if err else " (this rank succeeded)"))

    def info(self) -> dict:
        """bsg_comm_get_info: RCCL's rank count and this rank (ncclCommCount /
        ncclCommUserRank), the device, gathers issued and the graph cache's counters."""
        inf = self._nat.BsgCommInfo()
        self._nat.check_comm(self.lib.bsg_comm_get_info(self._comm, self._C.byref(inf)),
                             "bsg_comm_get_info")
        return {f: int(getattr(inf, f)) for f, _t in inf._fields_}

    def _stream(self):
        from .core import _raw_stream        # torch's raw current-stream handle (no Stream object)
        if _raw_stream is not None:
            return self._C.c_void_p(_raw_stream(self._dev))
        return self._C.c_void_p(torch.cuda.current_stream(self._dev).cuda_stream)

    def gather(self, out: torch.Tensor, src: torch.Tensor, slot: int):
        """out[world * src.numel()] <- every rank's src, on the comm's stream after the
        current stream's work; returns a handle whose wait() orders the current stream."""
        self._nat.check_comm(self.lib.bsg_comm_all_gather(
            self._comm, self._C.c_void_p(src.data_ptr()), self._C.c_void_p(out.data_ptr()),
            src.numel(), int(slot), self._stream()), "bsg_comm_all_gather")
        return _RcclWork(self, int(slot))

    def step_gather(self, batch, actions: torch.Tensor, rows: torch.Tensor, out: torch.Tensor,
                    slot: int):
        """bsg_step_gather: the wait for rows[slot]'s previous gather, the learner-row pointer,
        the step launch and this step's gather, in one C call (device spawns only).  Returns
        nothing: the caller keeps one work handle per slot (ShardedVectorEnv._rwork)."""
        a = actions
        if a.dtype is not torch.float64 or not a.is_contiguous() or a.device != batch.device:
            a = a.to(device=batch.device, dtype=torch.float64).contiguous()
        batch._keep = (a, None)
        batch.learner = rows
        C = self._C
        rc = self.lib.bsg_step_gather(batch._ctx, self._comm, C.c_void_p(a.data_ptr()), None,
                                      C.c_void_p(rows.data_ptr()), C.c_void_p(out.data_ptr()),
                                      slot, self._stream())
        if rc != 0:
            self._nat.check(rc, "bsg_step_gather")

    def wait(self, slot: int):
        self._nat.check_comm(self.lib.bsg_comm_wait(self._comm, int(slot), self._stream()),
                             "bsg_comm_wait")

    def all_reduce(self, t: torch.Tensor, avg: bool = True):
        """t (contiguous fp32 on this rank's device) <- the mean (avg) or sum over the ranks, in
        place: bsg_comm_all_reduce, ncclAllReduce on the current stream itself -- ordered
        with the kernels around it and recorded into a HIP graph when that stream is being
        captured (the C5 learner's gradient reduction, tools/sac_torch.py)."""
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device.type != "cuda":
            raise ValueError("all_reduce: a contiguous fp32 device tensor")
        op = self._nat.REDUCE_AVG if avg else self._nat.REDUCE_SUM
        self._nat.check_comm(self.lib.bsg_comm_all_reduce(
            self._comm, self._C.c_void_p(t.data_ptr()), t.numel(), op, self._stream()),
            "bsg_comm_all_reduce")

    def close(self):
        if self._comm is not None and self._comm.value:
            self.lib.bsg_comm_destroy(self._comm)
            self._comm = self._C.c_void_p()


class _RcclWork:
    def __init__(self, g, slot):
        self._g, self._slot = g, slot

    def wait(self):
        self._g.wait(self._slot)


class StaleRowsError(RuntimeError):
    """The gathered rows a Ready stands for were overwritten: their slot of the ring has been
    gathered into again since (ShardedVectorEnv.step)."""


class Ready:
    """Completion of one step's (or block's) gathered rows.  wait(): the current stream (RCCL)
    or the host (gloo) waits until every rank's rows of that step are in the gathered buffer.
    With an owner (ShardedVectorEnv) it also checks the rows are still there: the buffer is a
    ring of slots, and once the slot has been gathered into again wait() raises
    StaleRowsError instead of ordering the caller after rows that no longer exist."""

    __slots__ = ("_work", "_owner", "_slot", "_seq")

    def __init__(self, work=None, owner=None, slot=0, seq=0):
        self._work, self._owner, self._slot, self._seq = work, owner, slot, seq

    @property
    def valid(self) -> bool:
        """False once the rows' slot has been gathered into again."""
        return self._owner is None or self._owner._slot_seq[self._slot] == self._seq

    def wait(self):
        if not self.valid:
            raise StaleRowsError(
                f"gathered rows of gather #{self._seq} (slot {self._slot}) were overwritten by "
                f"gather #{self._owner._slot_seq[self._slot]}: a step's rows are valid for "
                f"{self._owner.rows_valid_steps} steps (ShardedVectorEnv.step)")
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
                 steps_per_gather: int = 1, transport="torch"):
        """collective: optional ``f(out, rows) -> Work`` that starts the gather of this
        rank's rows into ``out`` asynchronously (``Work.wait()`` = a stream wait), in place
        of RCCL's all_gather_into_tensor -- another transport, or a test's delayed copy
        (tests/test_gpu_sharded.py).  With it the overlapped path is used at any world size.
        transport: "torch" (torch.distributed's all_gather_into_tensor) or "rccl" (RcclGather:
        libbsg's direct RCCL calls, the low-host-overhead path; overlapped at any world
        size)."""
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
        self._collective = collective
        self._rccl = None
        if collective is None and transport == "rccl":
            self._rccl = RcclGather(dev, group)
        elif transport not in ("torch", "rccl"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = "rccl" if self._rccl is not None else ("custom" if collective else "torch")
        # the one-call step (bsg_step_gather): the Merge / Vertical / ... kinds with device
        # spawns (host-spawn rows and SectorCR's overflow note go through step_tensors)
        from . import _native as nat
        self._fused = (self._rccl is not None and self.k == 1
                       and getattr(self.local, "spawn_mode", "device") != "host"
                       and self.local.kind_cfg.kind != nat.ENV_SECTOR_CR)
        self.overlap = (collective is not None or self._rccl is not None
                        or (overlap and self.world > 1))
        # rows[blk, i]: the kernel's learner output of step i of block blk, a ring of R blocks:
        # R = BSG_COMM_SLOTS for the fused per-step gather (the step that rewrites a slot comes
        # R steps after its gather, which a fence the stream already waited for covers: one
        # stream wait per R/2 steps, bsg_comm.cpp), else 2
        R = nat.COMM_SLOTS if self._fused else 2
        self._nslots = R
        self._rows = torch.zeros((R, self.k, self.n_local, d), dtype=torch.float32, device=dev)
        self._gathered = torch.empty((R, self.world * self.k, self.n_local, d), dtype=torch.float32,
                                     device=dev)
        self._blk, self._i = 0, 0
        self._work = [None] * R
        # liveness: gathers issued, and the last one that wrote each slot (Ready.valid)
        self._gseq = 0
        self._slot_seq = [0] * R
        # the gather whose local rows a slot of self._rows holds now (-1 while a block is being
        # rewritten: the kernel starts overwriting a slot at the block's first step, up to k - 1
        # steps before the slot is gathered again; local_rows checks this)
        self._rows_seq = [0] * R
        self.rows_valid_steps = R * self.k
        if self._fused:
            # per slot, made once: the row block the kernel writes, the gathered view step()
            # returns and its completion work (the host side of a step is one C call)
            self._slot_rows = [self._rows[s, 0] for s in range(R)]
            self._views = [self._gathered[s].view(self.total_envs, d) for s in range(R)]
            self._rwork = [_RcclWork(self._rccl, s) for s in range(R)]

    def _slot(self):
        """Point the kernel's learner output at the next slot; before the first write into a
        block, wait (on the stream) for that block's previous gather."""
        blk, i = self._blk, self._i
        if i == 0:
            w = self._work[blk]
            if w is not None:
                w.wait()
                self._work[blk] = None
            elif self._fused:
                self._rccl.wait(blk)     # (a fused step's gather of this slot: no Work object)
            self._rows_seq[blk] = -1
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
        Ready); they may be read after ready.wait() for ``rows_valid_steps`` steps -- until
        their slot of the ring is gathered into again: BSG_COMM_SLOTS = 16 steps with the
        fused RCCL path (transport "rccl", device spawns), 2 otherwise.  k > 1: (None, None)
        inside a block, (block, Ready) at its last step; a block stays valid until the end of
        the next block (2k steps).  After that Ready.wait() raises StaleRowsError."""
        if self._fused:
            # transport "rccl", one gather per step, device spawns: one C call per step (the
            # wait for the slot's previous gather is libbsg's, bsg_step_gather)
            blk = self._blk
            self._rccl.step_gather(self.local.batch, local_actions, self._slot_rows[blk],
                                   self._gathered[blk], blk)
            self._blk = blk + 1 if blk + 1 < self._nslots else 0
            self._gseq += 1
            self._slot_seq[blk] = self._rows_seq[blk] = self._gseq
            return self._views[blk], Ready(self._rwork[blk], self, blk, self._gseq)
        blk, i = self._slot()
        self.local.step_tensors(local_actions)
        if i + 1 < self.k:
            self._i = i + 1
            return None, None
        return self._gather(blk, self.k)

    def local_rows(self, ready) -> torch.Tensor:
        """This rank's own learner rows behind a Ready ([n_local, obs+3] for k = 1, else
        [k, n_local, obs+3]): what every rank must find at this rank's place in the gathered
        rows (bench.py's cross-rank row check).  Raises StaleRowsError once the kernel has
        started rewriting them -- for k > 1 that is the first step of the slot's next block,
        before the slot is gathered again (the gathered rows stay valid until that gather)."""
        if not ready.valid or self._rows_seq[ready._slot] != ready._seq:
            raise StaleRowsError("the local rows of that gather were overwritten")
        blk = self._rows[ready._slot]
        return blk[0] if self.k == 1 else blk

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
            if self._rccl is not None:
                work = self._rccl.gather(out, src, blk)
            elif self._collective is not None:
                work = self._collective(out, src)
            else:
                work = all_gather_rows(out, src, self.group, async_op=True)
            self._work[blk] = work
        elif self.world == 1:
            out.copy_(src)
            work = None
        else:
            all_gather_rows(out, src, self.group)
            work = None
        self._gseq += 1
        self._slot_seq[blk] = self._rows_seq[blk] = self._gseq
        ready = Ready(work, self, blk, self._gseq)
        self._blk, self._i = (blk + 1) % self._nslots, 0
        if self.k == 1:
            return out.view(self.total_envs, self.row_dim), ready
        return out.view(self.world, n, self.n_local, self.row_dim).permute(1, 0, 2, 3), ready

    def close(self):
        for w in self._work:
            if w is not None:
                w.wait()
        self._work = [None] * self._nslots
        if self._rccl is not None:
            torch.cuda.synchronize(self.local.batch.device)
            self._rccl.close()
        self.local.close()
