"""Host-side cost per RL step of the N>1 bench path with a REAL ProcessGroupNCCL (RCCL)
all-gather, rehearsed on one GPU: a world-size-1 NCCL group whose all_gather_into_tensor
goes through the same torch/RCCL enqueue path (event records, Work objects, RCCL stream)
as on the 8-GPU node.  At 512 envs per GPU (C4's 8-GPU shard) the kernel is ~32 us, so
the host must enqueue a step in less than that or the node run is host-bound.

    python tools/shard_overhead_nccl.py            # E = 512 and 4096
Prints wall per step and host time per call for batch.step and ShardedVectorEnv.step, with
torch's all_gather_into_tensor and with libbsg's direct RCCL gather (transport="rccl").
"""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
import torch
import torch.distributed as dist

from bluesky_gym import parallel
from bluesky_gym.vector import MergeVectorEnv

T = 300


def timed(step):
    for k in range(30):
        step(k)
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for k in range(T):
        h0 = time.perf_counter()
        step(k)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / T * 1e6, host / T * 1e6


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    for E in (512, 4096):
        bank = torch.rand((16, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
        v = MergeVectorEnv(num_envs=E, num_ac=32, seed=1, compute_cd=True)
        v.reset()
        w, h = timed(lambda k: v.batch.step(bank[k % 16]))
        print(f"E={E:5d} plain batch.step              wall/step {w:7.1f} us  host/call {h:6.1f} us",
              flush=True)
        v.close()
        coll = lambda out, rows: dist.all_gather_into_tensor(out, rows, async_op=True)  # noqa: E731
        for K in (1, 8):
            s = parallel.ShardedVectorEnv(
                lambda **kw: MergeVectorEnv(num_ac=32, seed=1, compute_cd=True, **kw), E,
                collective=coll, steps_per_gather=K)
            s.reset()
            w, h = timed(lambda k: s.step(bank[k % 16]))
            print(f"E={E:5d} ShardedVectorEnv.step (RCCL, {K} step(s) per gather) wall/step {w:7.1f} us  "
                  f"host/call {h:6.1f} us", flush=True)
            if K == 8:
                break
            s.close()
        # libbsg's direct RCCL gather (parallel.RcclGather), one per step and per block of 8
        for graphs in ("1", "0"):
            os.environ["BSG_COMM_GRAPHS"] = graphs
            for K in (1, 8):
                r = parallel.ShardedVectorEnv(
                    lambda **kw: MergeVectorEnv(num_ac=32, seed=1, compute_cd=True, **kw), E,
                    steps_per_gather=K, transport="rccl")
                r.reset()
                w, h = timed(lambda k: r.step(bank[k % 16]))
                print(f"E={E:5d} ShardedVectorEnv.step (bsg_comm RCCL{' graph' if graphs == '1' else ''}, "
                      f"{K} step(s) per gather) wall/step {w:7.1f} us  host/call {h:6.1f} us", flush=True)
                if K == 1:
                    # the gather call alone (the step's rows of slot 0)
                    src, out = r._rows[0, 0], r._gathered[0][:1]
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in range(T):
                        r._rccl.gather(out, src, 0)
                    hg = (time.perf_counter() - t0) / T * 1e6
                    torch.cuda.synchronize()
                    print(f"E={E:5d}   bsg_comm_all_gather alone host/call {hg:6.1f} us", flush=True)
                r.close()
        # the enqueue cost of the collective alone
        out = torch.empty((E, s.local.batch.obs_dim + 3), dtype=torch.float32, device="cuda")
        rows = s._rows[0, 0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(T):
            dist.all_gather_into_tensor(out, rows, async_op=True)
        h = (time.perf_counter() - t0) / T * 1e6
        torch.cuda.synchronize()
        print(f"E={E:5d} all_gather_into_tensor alone  host/call {h:6.1f} us", flush=True)
        s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
