"""Which speculation condition of vert_own_fast fails (BSG_FAST_DEBUG build: the reason
mask lands in ep_info[:, 3]).  BSG_LIBRARY=.../libbsg_dbg.so python tools/fast_debug.py"""
import collections, os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import torch
from bluesky_gym import config, core
b = core.DeviceBatch(config.descent_config(), 4096, compute_cd=False, seed=1)
b.reset()
act = torch.rand((8, 4096, 1), dtype=torch.float64, device="cuda") * 2 - 1
hist = collections.Counter()
for k in range(250):
    b.ep_info[:, 3] = -1
    b.step(act[k % 8])
    w = b.ep_info[:, 3].cpu().numpy()
    for v in w:
        hist[int(v)] += 1
    if k in (5, 40, 120, 240):
        bad = (b.ep_info[:, 3] > 0).nonzero().flatten()[:3].tolist()
        for e in bad:
            print("env", e, {f: float(b.state[f][e, 0]) for f in ("alt", "hdg", "ap_trk", "selspd", "selalt", "selvs", "vs", "tas")})
print(sorted(hist.items()))
