"""Time the fused SAC actor kernel (bsg_policy_sac) over batch sizes: flat = per-workgroup
latency, linear = throughput.  python tools/policy_probe.py [tag]"""
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import torch  # noqa: E402
from bluesky_gym.policy import SACPolicy  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "descent"
pol = SACPolicy.from_npz(os.path.join("tests", "golden", "sac_actors.npz"), tag, "cuda")
for E in (16, 256, 1024, 4096, 16384, 65536):
    obs = torch.randn((E, pol.obs_dim), device="cuda")
    eps = torch.randn((E, pol.act_dim), device="cuda")
    out = torch.empty((E, pol.act_dim), dtype=torch.float64, device="cuda")
    for _ in range(20):
        pol(obs, eps, out=out)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    t0.record()
    for _ in range(n):
        pol(obs, eps, out=out)
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / n * 1e3
    gf = E * 2 * (pol.obs_dim * 256 + 256 * 256 + 2 * pol.act_dim * 256) / (us * 1e-6) / 1e12
    print(f"{tag} E={E:6d}: {us:8.2f} us per launch (back to back), {gf:6.1f} TFLOP/s", flush=True)
