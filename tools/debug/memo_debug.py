"""Debug: memo-valid vs memo-invalidated-every-launch vs no memo (Merge 128 x 32)."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd"), os.path.join(os.getcwd(), "tests")]
import torch
from bluesky_gym import config, core
from test_gpu_lookahead import _snap
sys.path.insert(0, os.path.join(os.getcwd(), "tools", "debug"))
from capture_debug import diff

def mk(memo=True, la=False, E=128, N=32):
    return core.DeviceBatch(config.merge_config(num_ac=N, max_episode_steps=20), E, compute_cd=True,
                            seed=5, learner=True, lookahead=la, memo_cache=memo)

def run(name, b, before=None, T=60):
    ref = mk()
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); b.reset()
    for t in range(T):
        a = torch.rand((128, 2), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        ref.step(a)
        if before: before(b, t)
        b.step(a)
        d = diff(_snap(ref), _snap(b))
        if d:
            print(f"  {name}: first diff at t={t}:", "; ".join(d[:6]))
            return
    print(f"  {name}: identical through t={T-1}")

run("no memo cache", mk(memo=False))
run("memo invalidated before every launch", mk(), before=lambda b, t: b.memo_cache.fill_(float("nan")))
run("memo invalidated from t=6", mk(), before=lambda b, t: b.memo_cache.fill_(float("nan")) if t >= 6 else None)
run("lookahead, memo invalidated from t=6", mk(la=True), before=lambda b, t: b.memo_cache.fill_(float("nan")) if t >= 6 else None)
