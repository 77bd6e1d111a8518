"""Per-wave phase cycles of the Descent 4096 step (stamps build, csrc `make stamps`) under
U(-1,1) actions or constant ones: where a launch's time goes.  GPU only:
  BSG_LIBRARY=.../libbsg_stamps.so python tools/probe/descent_stamps.py [uniform|descend]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import numpy as np
import torch

from bluesky_gym import config, core
from bluesky_gym import _native as nat

MODE = sys.argv[1] if len(sys.argv) > 1 else "uniform"
E = 4096
b = core.DeviceBatch(config.descent_config(), E, compute_cd=False, seed=1234,
                     autoreset=nat.AUTORESET_SAME_STEP, learner=True)
b.reset()
grid = E // 64
st = torch.zeros((2 * grid, 8), dtype=torch.int64, device="cuda")
nat.check(b.lib.bsg_set_stamps(b._ctx, C.c_void_p(st.data_ptr())), "bsg_set_stamps")
g = torch.Generator(device="cuda").manual_seed(3)
def act():
    if MODE == "descend":
        return torch.full((E, 1), -0.5, dtype=torch.float64, device="cuda")
    return torch.rand((E, 1), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
for k in range(60):
    b.step(act())
torch.cuda.synchronize()
recs = []
for k in range(40):
    st.zero_()
    b.step(act())
    torch.cuda.synchronize()
    recs.append(st[:grid].cpu().numpy().astype(np.int64))
r = np.concatenate(recs)
pct = lambda x: " ".join(f"{np.percentile(x, q):8.0f}" for q in (0, 10, 50, 90, 99, 100))
span = [(x[:, 6].max() - x[:, 0].min()) * 10 / 1000 for x in recs]
print(f"Descent E={E} actions={MODE}: kernel span (realtime, us) p50 {np.median(span):.1f} max {max(span):.1f}")
print("percentiles             0/10/50/90/99/100")
print("A spawn+substeps cyc", pct(r[:, 2] - r[:, 1]))
print("B obs cyc           ", pct(r[:, 3] - r[:, 2]))
print("rest cyc            ", pct(r[:, 5] - r[:, 3]))
print("total cycles        ", pct(r[:, 5] - r[:, 1]))
print("wave life us        ", pct((r[:, 6] - r[:, 0]) * 10 / 1000))
