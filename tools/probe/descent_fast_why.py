"""Descent 4096 under U(-1,1) actions (bench.py's env-only leg): how often vert_own_fast's
speculation fails, by reason bit (csrc/bsg_kernels.hip vert_own_fast `why`).  Needs the
debug build libbsg_fastdbg.so (make -C bluesky-gym-hallucination_amd/csrc OBJ_TAG=_fastdbg
CXXFLAGS_EXTRA=-DBSG_FAST_DEBUG=1 OUT=../bluesky_gym/_lib/libbsg_fastdbg.so), selected with
BSG_LIBRARY.  GPU only."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "bluesky-gym-hallucination_amd"))
from bluesky_gym import config, core  # noqa: E402

E = 4096
b = core.DeviceBatch(config.descent_config(), E, seed=0, compute_cd=False)
b.reset()
g = torch.Generator(device="cuda").manual_seed(1)
hist = {}
alts = []
STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 80
for t in range(STEPS):
    a = torch.rand((E, 1), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
    b.ep_info[:, 3] = 0.0
    pre = {k: b.state[k][:, 0].cpu().numpy().copy() for k in ("alt", "vs", "tas", "selalt", "selvs")}
    b.step(a)
    torch.cuda.synchronize()
    why = b.ep_info[:, 3].cpu().numpy().astype(np.int64)
    for e in np.nonzero(why)[0][:3]:
        print(f"step {t} env {e} why {why[e]} before: " +
              " ".join(f"{k}={pre[k][e]:.6g}" for k in pre) + f" action {float(a[e, 0]):.4f}")
    for w, c in zip(*np.unique(why, return_counts=True)):
        hist[int(w)] = hist.get(int(w), 0) + int(c)
    alts.append(b.state["alt"][:, 0].cpu().numpy())
tot = sum(hist.values())
print(f"why-code histogram over {STEPS} steps x 4096 envs (0 = fast path taken):")
for w in sorted(hist):
    print(f"  why={w:3d}  {hist[w]:8d}  {hist[w] / tot:.4f}")
alts = np.array(alts)
print("altitude percentiles (m):", np.percentile(alts, [0, 1, 50, 99, 100]).round(1).tolist())
print("share of env-steps at exactly 0 m:", float((alts == 0).mean()))
