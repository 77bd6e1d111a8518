import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import numpy as np, torch
from bluesky_gym import core, config
from oracle import batched as ob, bluesky_subset as bsx
E, N = 128, 32
b = core.DeviceBatch(config.vertical_config(num_intruders=N - 1), E, compute_cd=True, seed=99)
o = ob.VerticalOracle(E, num_ac=N, seed=99, compute_cd=True)
b.reset(); o.reset()
st0 = {f: b.state[f].cpu().numpy() for f in ("lat", "lon", "alt", "hdg", "tas", "vs", "cas")}
print("reset state maxdiff", {f: float(np.abs(st0[f] - getattr(o.st, f)).max()) for f in st0})
rng = np.random.default_rng(3)
a = rng.uniform(-1, 1, (E, 1))
b.step(torch.from_numpy(a)); r = o.step(a)
g = b.tcpamax.cpu().numpy(); ref = r["tcpamax"]
err = np.abs(g - ref) - (1e-5 + 1e-5 * np.abs(ref))
e, i = np.unravel_index(err.argmax(), err.shape)
print("worst", e, i, g[e, i], ref[e, i])
cd = r["cd"]
j = int(np.argmax(cd["tcpa"][e, i] * cd["swconfl"][e, i]))
print("argmax j", j, "tcpa", cd["tcpa"][e, i, j], "dist", cd["dist"][e, i, j])
st = {f: b.state[f].cpu().numpy() for f in ("lat", "lon", "alt", "hdg", "tas", "vs", "cas")}
cdg = bsx.statebased_detect(*(st[f][e:e+1] for f in ("lat", "lon", "alt", "hdg", "tas", "vs")))
print("gpu-state tcpa", cdg["tcpa"][0, i, j], "tcpamax", cdg["tcpamax"][0, i])
for f in st:
    print(f, st[f][e, [i, j]], getattr(o.st, f)[e, [i, j]], st[f][e, [i, j]] - getattr(o.st, f)[e, [i, j]])
print("spawn", o.device_spawn_params(np.array([e]), np.array([0]))[0][2 + 4 * (i - 1): 6 + 4 * (i - 1)] if i > 0 else None)
