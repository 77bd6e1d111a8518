"""Host time per call of each piece of one ShardedVectorEnv step on the overlapped RCCL
path (world-size-1 NCCL group on one GPU, as tools/shard_overhead_nccl.py): the Work.wait
of two steps ago, the learner-row pointer swap, the step launch (and its parts), the
all-gather enqueue.  Finds what to cut so that a C4 shard's host side stays below its
~30 us kernel.
    python tools/shard_host_breakdown.py [E] [steps_per_gather] [torch|rccl]
(rccl: libbsg's bsg_comm transport; BSG_COMM_PROFILE=1 adds the C call's own breakdown)
"""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29537")
import ctypes as C

import torch
import torch.distributed as dist

from bluesky_gym import parallel
from bluesky_gym.vector import MergeVectorEnv

T = 400


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    coll = lambda out, rows: dist.all_gather_into_tensor(out, rows, async_op=True)  # noqa: E731
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tr = sys.argv[3] if len(sys.argv) > 3 else "torch"
    s = parallel.ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=1, compute_cd=True, **kw),
                                  E, collective=coll if tr == "torch" else None, steps_per_gather=K,
                                  transport=tr)
    s.reset()
    b = s.local.batch
    bank = torch.rand((16, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
    views = [bank[k] for k in range(16)]
    acc = {}

    def tick(name, t0):
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0

    for k in range(32):
        s.step(views[k % 16])
    s.flush()
    torch.cuda.synchronize()
    acc.clear()
    t_all = time.perf_counter()
    for k in range(T):
        t0 = time.perf_counter()
        x = bank[k % 16]
        tick("bank[k] view", t0)
        t0 = time.perf_counter()
        blk, i = s._slot()
        tick("_slot (Work.wait + set_learner)", t0)
        t0 = time.perf_counter()
        st = torch.cuda.current_stream(b.device).cuda_stream
        tick("  torch.cuda.current_stream", t0)
        t0 = time.perf_counter()
        s.local.step_tensors(x)
        tick("step_tensors", t0)
        t0 = time.perf_counter()
        if i + 1 < s.k:
            s._i = i + 1
        else:
            s._gather(blk, s.k)
        tick("_gather (all_gather enqueue)", t0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) / T * 1e6
    for n, v in acc.items():
        print(f"E={E} k={K} {tr} {n:32s} {v / T * 1e6:7.2f} us/call", flush=True)
    print(f"E={E} k={K} {tr} wall per step {wall:.1f} us (incl. the instrumentation)", flush=True)
    t0 = time.perf_counter()
    for k in range(T):
        b.lib.bsg_abi_version()
    print(f"E={E} bare ctypes call {(time.perf_counter() - t0) / T * 1e6:.2f} us", flush=True)
    s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
