"""Debug: first conf_mask mismatch of the wind batch parity (P points) -- prints the
oracle's StateBased terms for the mismatching pairs and the device/oracle state gap."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
from oracle import batched as ob
from oracle import bluesky_subset as bsx
from bluesky_gym import config, core
from bluesky_gym.wind import WindTable

P = int(sys.argv[1]) if len(sys.argv) > 1 else 12
auto = int(sys.argv[2]) if len(sys.argv) > 2 else 2
E, N, T = 128, 32, 60
rng = np.random.default_rng(P)
lat = rng.uniform(52.3, 54.3, P); lon = rng.uniform(3.8, 5.6, P)
vn, ve = rng.uniform(-20, 20, (1, P)), rng.uniform(-20, 20, (1, P))
b = core.DeviceBatch(config.merge_config(num_ac=N), E, autoreset=auto, compute_cd=True, seed=77)
b.set_wind(WindTable(lat, lon, vn, ve), augment_obs=True)
o = ob.MergeOracle(E, num_ac=N, autoreset=auto, seed=77, compute_cd=True)
f = bsx.WindField(); f.addpointvne(lat, lon, vn, ve)
o.set_wind(f, augment_obs=True)
b.reset(); o.reset()
ra = np.random.default_rng(3)
for t in range(T):
    a = ra.uniform(-1, 1, (E, 2))
    b.step(torch.from_numpy(a))
    r = o.step(a)
    for fld in ("lat", "lon", "hdg", "trk", "gs", "tas"):
        d = np.abs(b.state[fld].cpu().numpy() - getattr(o.st, fld))
        if fld in ("hdg", "trk"):
            d = np.minimum(d, 360 - d)
        print(t, fld, "maxdiff", d.max(), "nexact", (d == 0).mean())
    cm = b.conf_mask.cpu().numpy().astype(np.uint64)
    bad = np.argwhere(cm != r["conf_mask"])
    if len(bad):
        cd = r["cd"]
        for e, i in bad[:4]:
            x = int(cm[e, i]) ^ int(r["conf_mask"][e, i])
            for k in range(N):
                if (x >> k) & 1:
                    print("env", e, "pair", i, k, "dev", (int(cm[e, i]) >> k) & 1,
                          "dcpa2-R2", cd["dcpa2"][e, i, k] - bsx.RPZ ** 2,
                          "tin", cd["tinconf"][e, i, k], "tout", cd["toutconf"][e, i, k],
                          "tcpa", cd["tcpa"][e, i, k], "dist", cd["dist"][e, i, k])
        break
