"""Per-wave phase timing from the diagnostic build (make -C .../csrc stamps).

Run on the GPU box:  BSG_LIBRARY=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_stamps.so \
                     python tools/stamps.py [E] [N]
"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import numpy as np
import torch

from bluesky_gym import config, core
from bluesky_gym import _native as nat

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 32
b = core.DeviceBatch(config.merge_config(num_ac=N), E, compute_cd=True, seed=1234)
b.reset()
gs = 1
while gs < N:
    gs <<= 1
grid = (E + 64 // gs - 1) // (64 // gs)
st = torch.zeros((grid, 8), dtype=torch.int64, device="cuda")
nat.check(b.lib.bsg_set_stamps(b._ctx, C.c_void_p(st.data_ptr())), "bsg_set_stamps")
act = torch.rand((8, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
for k in range(30):
    b.step(act[k % 8])
torch.cuda.synchronize()
recs = []
for k in range(5):
    st.zero_()
    b.step(act[k % 8])
    torch.cuda.synchronize()
    recs.append(st.cpu().numpy().astype(np.uint64))
r = np.concatenate(recs)
rt0 = r[:, 0].astype(np.int64); rt1 = r[:, 6].astype(np.int64)
c1 = r[:, 1].astype(np.int64); c2 = r[:, 2].astype(np.int64); c3 = r[:, 3].astype(np.int64)
c4 = (r[:, 4] & np.uint64((1 << 48) - 1)).astype(np.int64); tot = (r[:, 4] >> np.uint64(48)).astype(np.int64)
c5 = r[:, 5].astype(np.int64)
pct = lambda x: " ".join(f"{np.percentile(x, q):8.0f}" for q in (0, 10, 50, 90, 99, 100))
print(f"E={E} N={N} grid={grid}  (percentiles 0/10/50/90/99/100)")
for run in range(5):
    s = slice(run * grid, (run + 1) * grid)
    print(f"run {run}: kernel span (realtime) {(rt1[s].max() - rt0[s].min()) * 10 / 1000:.1f} us, "
          f"start spread {(rt0[s].max() - rt0[s].min()) * 10 / 1000:.2f} us")
print("wave life (us)      ", pct((rt1 - rt0) * 10 / 1000 * 1000))
print("A spawn+substeps cyc", pct(c2 - c1))
print("B obs+rank cyc      ", pct(c3 - c2))
print("CD phase1 cyc       ", pct(c4 - c3))
print("CD phase2+out cyc   ", pct(c5 - c4))
print("candidates/wave     ", pct(tot))
print("total cycles        ", pct(c5 - c1))
hw = r[:, 7].astype(np.int64)
print("xcc ids seen", np.unique(hw)[:16])
