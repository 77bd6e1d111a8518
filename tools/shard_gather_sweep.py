"""Wall time per step of the fused per-step gather (ShardedVectorEnv, transport "rccl",
k = 1: bsg_step_gather) at C4's shard sizes, beside the bare launch loop and torch's
all_gather_into_tensor per step.  One GPU, a world-size-1 RCCL group (the node's enqueue
path; the gather's bytes never leave the GPU, so this measures the per-step overhead).

    python tools/shard_gather_sweep.py [E ...]
"""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
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
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    sizes = [int(x) for x in sys.argv[1:]] or [512, 1024, 2048, 4096]
    for E in sizes:
        bank = torch.rand((16, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
        v = MergeVectorEnv(num_envs=E, num_ac=32, seed=1, compute_cd=True)
        v.reset()
        w, h = timed(lambda k: v.batch.step(bank[k % 16]))
        print(f"E={E:5d} batch.step (no gather)             wall/step {w:7.1f} us  host/call {h:6.1f} us", flush=True)
        v.close()
        coll = lambda out, rows: dist.all_gather_into_tensor(out, rows, async_op=True)  # noqa: E731
        for transport in ("rccl", "torch"):
            r = parallel.ShardedVectorEnv(
                lambda **kw: MergeVectorEnv(num_ac=32, seed=1, compute_cd=True, **kw), E,
                steps_per_gather=1, transport=transport,
                collective=coll if transport == "torch" else None)
            r.reset()
            w, h = timed(lambda k: r.step(bank[k % 16]))
            name = "fused step+gather (libbsg)   " if transport == "rccl" else "step + torch all_gather (RCCL)"
            print(f"E={E:5d} {name}   wall/step {w:7.1f} us  host/call {h:6.1f} us", flush=True)
            r.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
