"""Per-launch kernel times (HIP event pair around every launch) of DescentEnv batches, to
compare the specialised ownship loop with substep() (BSG_NO_FASTPATH=1):
    python tools/descent_timing.py [kind]"""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import numpy as np
import torch
from bluesky_gym import config, core

kind = sys.argv[1] if len(sys.argv) > 1 else "descent"
for E in (512, 1024, 2048, 4096):
    for nf in ("0", "1"):
        os.environ["BSG_NO_FASTPATH"] = nf
        cfg = config.descent_config() if kind == "descent" else config.vertical_config(num_intruders=31)
        b = core.DeviceBatch(cfg, E, compute_cd=kind != "descent", seed=1)
        b.reset()
        act = torch.rand((8, E, 1), dtype=torch.float64, device="cuda") * 2 - 1
        for k in range(10):
            b.step(act[k % 8])
        torch.cuda.synchronize()
        ts = []
        for k in range(100):
            b.set_timing(1)
            b.step(act[k % 8])
            torch.cuda.synchronize()
            ms, n = b.step_timing()
            ts.append(ms * 1e3 / n)
        b.set_timing(0)
        ts = np.array(ts)
        print(f"{kind} E={E:5d} {'general' if nf == '1' else 'fast   '} min {ts.min():6.1f} "
              f"p50 {np.median(ts):6.1f} p90 {np.percentile(ts, 90):6.1f} max {ts.max():6.1f} us",
              flush=True)
        b.close()
