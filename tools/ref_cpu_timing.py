"""Container-only timing of the REFERENCE env code on CPU (never runs on the GPU box).

Drives the reference's own MergeEnv (merge_env.py, stub-imported by oracle/ref_harness.py,
`bluesky` bound to the NumPy BlueSky-subset restatement) one env in one process -- the
reference's layout (one env per SubprocVecEnv worker) -- and, on the same core, the batched
NumPy port (oracle/batched.py) that bench.py's cpu_baseline times on the GPU box:

    python tools/ref_cpu_timing.py [num_ac] [seconds]
"""
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import batched as ob                     # noqa: E402
from oracle.ref_harness import load_reference_envs  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
SEC = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0

bs, mods = load_reference_envs()
m = mods["merge"]
m.NUM_AC = N
random.seed(0)
env = m.MergeEnv()
rng = np.random.default_rng(0)
env.reset()
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < SEC:
    obs, r, term, trunc, info = env.step(rng.uniform(-1, 1, 2))
    n += 1
    if term or n % 50 == 0:
        env.reset()
ref = n / (time.perf_counter() - t0)

E = 128
o = ob.MergeOracle(E, num_ac=N, seed=1, compute_cd=True)
o.reset()
k, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < SEC:
    o.step(rng.uniform(-1, 1, (E, 2)))
    k += 1
port = E * k / (time.perf_counter() - t0)
cpu = "unknown"
with open("/proc/cpuinfo") as f:
    for line in f:
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
print(f"MergeEnv-v0 N={N}, one core of '{cpu}':")
print(f"  reference env code (merge_env.py + NumPy BlueSky subset, 1 env): {ref:8.1f} env-steps/s")
print(f"  batched NumPy port (oracle/batched.py, {E} envs, StateBased CD on): {port:8.1f} env-steps/s")
