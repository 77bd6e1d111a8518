"""Kernel trace helper for the fused per-step gather at one shard size (run under
rocprofv3 --kernel-trace): python tools/gather_trace.py E [steps] [mode]
mode: fused (ShardedVectorEnv, transport rccl, k = 1) | bare (batch.step only)"""
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
import torch
import torch.distributed as dist

from bluesky_gym import parallel
from bluesky_gym.vector import MergeVectorEnv

E = int(sys.argv[1])
T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
mode = sys.argv[3] if len(sys.argv) > 3 else "fused"
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
bank = torch.rand((16, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
if mode == "bare":
    v = MergeVectorEnv(num_envs=E, num_ac=32, seed=1, compute_cd=True)
    v.reset()
    step = lambda k: v.batch.step(bank[k % 16])  # noqa: E731
else:
    v = parallel.ShardedVectorEnv(lambda **kw: MergeVectorEnv(num_ac=32, seed=1, compute_cd=True, **kw),
                                  E, steps_per_gather=1, transport="rccl")
    v.reset()
    step = lambda k: v.step(bank[k % 16])  # noqa: E731
import time
for k in range(50):
    step(k)
torch.cuda.synchronize()
h = 0.0
t0 = time.perf_counter()
for k in range(T):
    h0 = time.perf_counter()
    step(k)
    h += time.perf_counter() - h0
torch.cuda.synchronize()
print(f"{mode} E={E}: wall/step {(time.perf_counter() - t0) / T * 1e6:.1f} us, host/call {h / T * 1e6:.1f} us", flush=True)
v.close()
dist.destroy_process_group()
print("done", mode, E, T)
