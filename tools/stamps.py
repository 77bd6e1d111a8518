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
KIND = os.environ.get("STAMPS_KIND", "merge")      # merge | vertical
cfg = (config.merge_config(num_ac=N) if KIND == "merge"
       else config.vertical_config(num_intruders=N - 1))
b = core.DeviceBatch(cfg, E, compute_cd=True, seed=1234)
b.reset()
gs = 1
while gs < N:
    gs <<= 1
grid = (E + 64 // gs - 1) // (64 // gs)
# (x2: with the lookahead on (E <= 2048) its extra workgroups, blockIdx >= grid, stamp
# slots 0-1 before they branch off; their rows are ignored below)
st = torch.zeros((2 * grid, 8), dtype=torch.int64, device="cuda")
nat.check(b.lib.bsg_set_stamps(b._ctx, C.c_void_p(st.data_ptr())), "bsg_set_stamps")
act = torch.rand((8, E, b.act_dim), dtype=torch.float64, device="cuda") * 2 - 1
for k in range(30):
    b.step(act[k % 8])
torch.cuda.synchronize()
recs = []
la_recs = []
feats = []
FIX = (config.FIX_LAT, config.FIX_LON)
for k in range(5):
    st.zero_()
    pre = {f: b.state[f].cpu().numpy().copy() for f in ("lat", "lon", "hdg", "tas", "nav", "alt")}
    flags = b.envs["flags"].cpu().numpy().copy()
    b.step(act[k % 8])
    torch.cuda.synchronize()
    recs.append(st[:grid].cpu().numpy().astype(np.uint64))
    la_recs.append(st[grid:].cpu().numpy().astype(np.uint64))
    post = {f: b.state[f].cpu().numpy() for f in ("lat", "lon", "hdg", "tas", "nav")}
    # per-lane features of this step, folded per wave (64/gs envs per wave)
    wp = np.where(((pre["nav"] >> 8) & 255) == 0, FIX[0], config.RWY_LAT)
    wpn = np.where(((pre["nav"] >> 8) & 255) == 0, FIX[1], config.RWY_LON)
    dlat = np.radians(wp - pre["lat"]); dlon = np.radians(wpn - pre["lon"])
    dkm = 6371.0 * np.sqrt(dlat ** 2 + (dlon * np.cos(np.radians(pre["lat"]))) ** 2)
    lnav = (pre["nav"] & 1) == 1
    near = lnav & (dkm < 40.0)
    switched = ((post["nav"] >> 8) & 255) != ((pre["nav"] >> 8) & 255)
    lnav_off = lnav & ((post["nav"] & 1) == 0)
    dh = np.abs(((post["hdg"] - pre["hdg"] + 180) % 360) - 180)
    turning = dh > 1.0
    spd = np.abs(post["tas"] - pre["tas"]) > 1e-9
    epw = 64 // gs
    def per_wave(x):
        x = np.asarray(x, np.float64).reshape(-1, N).sum(1)
        pad = (-len(x)) % epw
        return np.concatenate([x, np.zeros(pad)]).reshape(-1, epw).sum(1)
    feats.append(np.stack([per_wave(near), per_wave(switched | lnav_off), per_wave(turning),
                           per_wave(spd), per_wave(np.repeat(flags & 1, N).reshape(-1, N)),
                           per_wave(lnav)], 1))
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
F = np.concatenate(feats)
A = (c2 - c1).astype(np.float64)
names = ["lanes near wp (<40km)", "lanes wp switch/off", "lanes turning >1deg", "lanes speed change",
         "lanes resetting", "lanes LNAV"]
print("phase-A cycles vs per-wave features (Pearson r, mean of feature, A p50 for feature==0 / >0):")
for i, nm in enumerate(names):
    x = F[:, i]
    r_ = np.corrcoef(x, A)[0, 1] if x.std() > 0 else float("nan")
    a0 = np.median(A[x == 0]) if (x == 0).any() else float("nan")
    a1 = np.median(A[x > 0]) if (x > 0).any() else float("nan")
    print(f"  {nm:24s} r={r_:+.2f} mean={x.mean():6.2f}  A|0={a0:9.0f}  A|>0={a1:9.0f}")
hw = r[:, 7].astype(np.uint64)
xcc = (hw >> np.uint64(32)).astype(np.int64)
hid = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
simd = (hid >> 4) & 3
cu = (hid >> 8) & 15
sh = (hid >> 12) & 1
se = (hid >> 13) & 7
print("xcc ids seen", np.unique(xcc)[:16])
life = (rt1 - rt0) * 10 / 1000
tot_c = c5 - c1
for run in range(5):
    s = slice(run * grid, (run + 1) * grid)
    key = (((xcc[s] * 8 + se[s]) * 2 + sh[s]) * 16 + cu[s]) * 4 + simd[s]
    cuk = key // 4
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    per_wave = cnt[inv]
    ucu, cinv, ccnt = np.unique(cuk, return_inverse=True, return_counts=True)
    print(f"run {run}: {len(uk)} SIMDs used, waves/SIMD histogram",
          dict(zip(*np.unique(cnt, return_counts=True))), f"; {len(ucu)} CUs, waves/CU",
          dict(zip(*np.unique(ccnt, return_counts=True))))
    for w in sorted(set(per_wave.tolist())):
        sel = per_wave == w
        print(f"   waves sharing a SIMD={w}: n={sel.sum():5d}  life us p50 {np.median(life[s][sel]):6.1f} "
              f"max {life[s][sel].max():6.1f}   cycles p50 {np.median(tot_c[s][sel]):8.0f} "
              f"max {tot_c[s][sel].max():8.0f}")
# per-SIMD pairs (run 0..4): the earlier- and later-finishing wave of each 2-wave SIMD and
# their wave slot ids (HW_ID bits 3:0) -- tests the age-priority arbitration hypothesis
slot = hid & 15
first_l, second_l, first_s, second_s, start_gap = [], [], [], [], []
for run in range(5):
    s = np.arange(run * grid, (run + 1) * grid)
    key = (((xcc[s] * 8 + se[s]) * 2 + sh[s]) * 16 + cu[s]) * 4 + simd[s]
    order = np.argsort(key, kind="stable")
    ks = key[order]
    for i in range(len(ks) - 1):
        if ks[i] == ks[i + 1] and (i == 0 or ks[i - 1] != ks[i]) and (i + 2 >= len(ks) or ks[i + 2] != ks[i]):
            a, bb = s[order[i]], s[order[i + 1]]
            if rt1[a] > rt1[bb]:
                a, bb = bb, a
            first_l.append(life[a]); second_l.append(life[bb])
            first_s.append(slot[a]); second_s.append(slot[bb])
            start_gap.append((rt0[bb] - rt0[a]) * 10 / 1000)
first_l = np.array(first_l); second_l = np.array(second_l)
print("2-wave SIMDs:", len(first_l))
if len(first_l) == 0:
    first_l = second_l = np.zeros(1)
    start_gap, first_s, second_s = [0.0], [0], [0]
print("  first-finishing wave life ns ", pct(first_l * 1000))
print("  second-finishing wave life ns", pct(second_l * 1000))
print("  start(second) - start(first) ns", pct(np.array(start_gap) * 1000))
print("  slot pairs (first,second) most common:",
      sorted(zip(*np.unique(np.stack([first_s, second_s], 1), axis=0, return_counts=True)),
             key=lambda t: -t[1])[:6])

# what sets the kernel span: per-SIMD finish times (last wave's end - kernel start) and the
# phases / features of the waves on the latest-finishing SIMDs
print("per-SIMD finish (us after the first wave start), percentiles 50/90/99/99.9/100, and the "
      "5 latest SIMDs' waves (A, B, CD1, CD2 kcycles; near, switch, turning, speed, resetting lanes; "
      "CD candidates):")
for run in range(1, 5):
    s = np.arange(run * grid, (run + 1) * grid)
    key = (((xcc[s] * 8 + se[s]) * 2 + sh[s]) * 16 + cu[s]) * 4 + simd[s]
    t0k = rt0[s].min()
    uk, inv = np.unique(key, return_inverse=True)
    fin = np.zeros(len(uk), np.int64)
    np.maximum.at(fin, inv, rt1[s] - t0k)
    fin_us = fin * 10 / 1000
    q = " ".join(f"{np.percentile(fin_us, p):6.1f}" for p in (50, 90, 99, 99.9, 100))
    print(f" run {run}: {q}")
    for j in np.argsort(fin)[-5:][::-1]:
        ws = s[inv == j]
        desc = []
        for w in ws:
            desc.append(f"[A {(c2[w]-c1[w])/1e3:5.1f} B {(c3[w]-c2[w])/1e3:4.1f} CD1 {(c4[w]-c3[w])/1e3:4.1f} "
                        f"CD2 {(c5[w]-c4[w])/1e3:4.1f} | {' '.join(str(int(v)) for v in F[w, :5])} | cand {tot[w]}]")
        print(f"   SIMD fin {fin_us[j]:5.1f} us: " + " ".join(desc))

# lookahead workgroups (E <= 2048: blockIdx >= grid), if any ran: their life against the
# main waves' (realtime stamps, 100 MHz)
la = np.concatenate(la_recs)
ran = la[:, 0] != 0
if ran.any():
    lr0 = la[ran, 0].astype(np.int64); lr1 = la[ran, 6].astype(np.int64)
    print("lookahead waves: n per launch", int(ran.sum()) // 5, " life (us)", pct((lr1 - lr0) * 10 / 1000 * 1000))
    lc1 = la[ran, 1].astype(np.int64); lc2 = la[ran, 2].astype(np.int64); lc3 = la[ran, 3].astype(np.int64)
    nr = la[ran, 4].astype(np.int64)
    lr = (lr1 - lr0) * 10 / 1000
    ok = (lc2 != 0) & (lc3 != 0)
    for nm, sel in (("no resetting lane", ok & (nr == 0)), ("resetting lanes", ok & (nr > 0))):
        if sel.any():
            print(f"lookahead waves, {nm}: n={int(sel.sum())}  life us {pct(lr[sel] * 1000)}")
            print(f"   entry -> propagate (loads, spawn) cyc {pct(lc2[sel] - lc1[sel])}")
            print(f"   propagate cyc                         {pct(lc3[sel] - lc2[sel])}")
            lc5 = la[ran, 5].astype(np.int64); cr = la[ran, 7].astype(np.int64)
            s5 = sel & (lc5 != 0)
            if s5.any():
                print(f"   first substep cyc                     {pct(lc5[s5] - lc2[s5])}")
                print(f"   substeps 2.. cyc                      {pct(lc3[s5] - lc5[s5])}")
                print(f"   cruise loop: {int((cr[s5] == 1).sum())} of {int(s5.sum())} waves")
    for run in range(1, 5):
        s_ = slice(run * grid, (run + 1) * grid)
        t0k = rt0[s_].min()
        lm = la[run * grid:(run + 1) * grid]
        lm = lm[lm[:, 0] != 0]
        print(f" run {run}: main waves end {(rt1[s_].max() - t0k) * 10 / 1000:.1f} us, "
              f"lookahead waves end {(lm[:, 6].astype(np.int64).max() - t0k) * 10 / 1000:.1f} us after the first start")
