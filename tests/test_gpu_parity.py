"""GPU parity: libbsg.so (HIP, gfx950) against the CPU oracle and the golden vectors.

Bar (BASELINE.json north_star): bit-exact for booleans and indices (terminated,
truncated, top-K intruder indices, intrusion masks, StateBased conflict / LoS masks);
fp32 observations and rewards within |gpu - ref| <= 1e-5 + 1e-5 * |ref|.
"""
import numpy as np
import pytest
import torch

import oracle_replay as rp
from oracle import batched as ob

pytestmark = pytest.mark.gpu

ATOL = 1e-5
RTOL = 1e-5
GOLD = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden")


# tcpa of an exactly parallel, equal-speed pair is ill-conditioned: its relative velocity
# is rounding noise (|dv| ~ 1e-13 m/s), StateBased floors dv2 at 1e-6 and tcpa becomes
# noise of order |dv|*dist/1e-6 <= ~0.1 s (creconfs intruders with equal dpsi hit this).
# The conflict / LoS masks of such pairs are robust and stay bit-exact.
TCPA_ATOL = 0.1


def close(a, b, what, atol=ATOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + RTOL * np.abs(b))
    assert np.all(np.isfinite(a)), what + ": non-finite"
    assert err.max(initial=-1) <= 0, f"{what}: max excess {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"


def bits(mask_u64, n):
    m = np.asarray(mask_u64).astype(np.uint64)
    return np.stack([(m >> np.uint64(i)) & np.uint64(1) for i in range(n)], -1).astype(np.int8)


@pytest.fixture(scope="module")
def bg():
    from bluesky_gym import core, config, _native
    return core, config, _native


def load(name):
    return dict(np.load(f"{GOLD}/{name}.npz"))


@pytest.mark.parametrize("name", ["merge_N8", "merge_N16", "merge_N20", "merge_N32"])
def test_merge_golden_on_gpu(bg, name):
    core, config, nat = bg
    g = load(name)
    n_ep, T = g["actions"].shape[:2]
    N = int(g["num_ac"])
    b = core.DeviceBatch(config.merge_config(num_ac=N), n_ep, autoreset=nat.AUTORESET_NONE,
                         compute_cd=True)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    m = rp.step_mask(g)
    act = torch.from_numpy(g["actions"]).cuda()
    for t in range(T):
        obs, rew, term, trunc = b.step(act[:, t])
        live = m[:, t]
        if not live.any():
            break
        close(obs.cpu().numpy()[live], g["obs"][live, t], f"obs t={t}")
        close(rew.cpu().numpy()[live], g["reward"][live, t], f"reward t={t}")
        assert np.array_equal(term.cpu().numpy()[live], g["terminated"][live, t].astype(np.uint8)), t
        assert np.array_equal(trunc.cpu().numpy()[live], g["truncated"][live, t].astype(np.uint8)), t
        assert np.array_equal(b.topk.cpu().numpy()[live], g["topk"][live, t]), t
        ib = bits(b.intr_mask.cpu().numpy(), N)[:, 1:]
        assert np.array_equal(ib[live], g["intr"][live, t]), t


@pytest.mark.parametrize("name", ["vertical_N6", "vertical_N32"])
def test_vertical_golden_on_gpu(bg, name):
    core, config, nat = bg
    g = load(name)
    n_ep, T = g["actions"].shape[:2]
    N = int(g["num_ac"])
    b = core.DeviceBatch(config.vertical_config(num_intruders=N - 1), n_ep,
                         autoreset=nat.AUTORESET_NONE, compute_cd=True)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    m = rp.step_mask(g)
    act = torch.from_numpy(g["actions"]).cuda()
    for t in range(T):
        obs, rew, term, trunc = b.step(act[:, t])
        live = m[:, t]
        if not live.any():
            break
        close(obs.cpu().numpy()[live], g["obs"][live, t], f"obs t={t}")
        close(rew.cpu().numpy()[live], g["reward"][live, t], f"reward t={t}")
        assert np.array_equal(term.cpu().numpy()[live], g["terminated"][live, t].astype(np.uint8)), t
        nt = live & (g["terminated"][:, t] == 0)
        ib = bits(b.intr_mask.cpu().numpy(), N)[:, 1:]
        assert np.array_equal(ib[nt], g["intr"][nt, t]), t


def test_descent_golden_on_gpu(bg):
    core, config, nat = bg
    g = load("descent")
    n_ep, T = g["actions"].shape[:2]
    b = core.DeviceBatch(config.descent_config(), n_ep, autoreset=nat.AUTORESET_NONE)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    m = rp.step_mask(g)
    act = torch.from_numpy(g["actions"]).cuda()
    for t in range(T):
        obs, rew, term, trunc = b.step(act[:, t])
        live = m[:, t]
        if not live.any():
            break
        close(obs.cpu().numpy()[live], g["obs"][live, t], f"obs t={t}")
        close(rew.cpu().numpy()[live], g["reward"][live, t], f"reward t={t}")
        assert np.array_equal(term.cpu().numpy()[live], g["terminated"][live, t].astype(np.uint8)), t


@pytest.mark.parametrize("name", ["horizontal_N6", "horizontal_N16"])
def test_horizontal_golden_on_gpu(bg, name):
    core, config, nat = bg
    g = load(name)
    n_ep, T = g["actions"].shape[:2]
    N = int(g["num_ac"])
    b = core.DeviceBatch(config.horizontal_config(num_intruders=N - 1), n_ep,
                         autoreset=nat.AUTORESET_NONE, compute_cd=True)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    wpt = np.stack([b.envs["env_wpt_lat"].cpu().numpy(), b.envs["env_wpt_lon"].cpu().numpy()], 1)
    assert np.array_equal(wpt, g["wpt"])
    m = rp.step_mask(g)
    act = torch.from_numpy(g["actions"]).cuda()
    for t in range(T):
        obs, rew, term, trunc = b.step(act[:, t])
        live = m[:, t]
        if not live.any():
            break
        close(obs.cpu().numpy()[live], g["obs"][live, t], f"obs t={t}")
        close(rew.cpu().numpy()[live], g["reward"][live, t], f"reward t={t}")
        assert np.array_equal(term.cpu().numpy()[live], g["terminated"][live, t].astype(np.uint8)), t
        assert np.array_equal(trunc.cpu().numpy()[live], g["truncated"][live, t].astype(np.uint8)), t
        nt = live & (g["terminated"][:, t] == 0)
        ib = bits(b.intr_mask.cpu().numpy(), N)[:, 1:]
        assert np.array_equal(ib[nt], g["intr"][nt, t]), t


def _compare_step(b, r, N, kind, t):
    close(b.obs.cpu().numpy(), r["obs"], f"obs t={t}")
    close(b.reward.cpu().numpy(), r["reward"], f"reward t={t}")
    assert np.array_equal(b.terminated.cpu().numpy().astype(bool), r["terminated"]), t
    assert np.array_equal(b.truncated.cpu().numpy().astype(bool), r["truncated"]), t
    if kind != "descent":
        # reset steps included: the reset observation's top-K and an intrusion mask of 0
        gi = b.intr_mask.cpu().numpy().astype(np.uint64)
        assert np.array_equal(gi, r["intr_mask"]), t
        assert np.array_equal(b.conf_mask.cpu().numpy().astype(np.uint64), r["conf_mask"]), t
        assert np.array_equal(b.los_mask.cpu().numpy().astype(np.uint64), r["los_mask"]), t
        close(b.tcpamax.cpu().numpy(), r["tcpamax"], f"tcpamax t={t}", atol=TCPA_ATOL)
        ms_g = b.min_sep.cpu().numpy().astype(np.float64)
        ms_r = r["min_sep"]
        assert np.array_equal(np.isinf(ms_g), np.isinf(ms_r)), t
        fin = np.isfinite(ms_r)
        close(ms_g[fin], ms_r[fin], f"min_sep t={t}")
    if kind == "merge":
        assert np.array_equal(b.topk.cpu().numpy(), r["topk"]), t


@pytest.mark.parametrize("autoreset", [ob.AUTORESET_NEXT_STEP, ob.AUTORESET_SAME_STEP])
def test_merge_batch_autoreset_parity(bg, autoreset):
    """256 envs x 32 aircraft, device Philox spawns, random actions, 120 steps (two full
    TimeLimit episodes plus early terminations): every output vs the oracle."""
    core, config, nat = bg
    E, N, T = 256, 32, 120
    seed = 1234
    b = core.DeviceBatch(config.merge_config(num_ac=N), E, autoreset=autoreset,
                         compute_cd=True, seed=seed)
    o = ob.MergeOracle(E, num_ac=N, autoreset=autoreset, seed=seed, compute_cd=True)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(7)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, N, "merge", t)
        if autoreset == ob.AUTORESET_SAME_STEP and r["final_obs"] is not None:
            d = r["terminated"] | r["truncated"]
            close(b.final_obs.cpu().numpy()[d], r["final_obs"][d], f"final_obs t={t}")


PATCHED = {"D_HEADING": 30.0, "INTRUSION_DISTANCE": 9.0, "DISTANCE_MARGIN": 25.0,
           "DRIFT_PENALTY": -0.25, "INTRUDER_DISTANCE_MAX": 150.0}


@pytest.mark.parametrize("lookahead", [True, False])
def test_merge_patched_constants_parity(bg, lookahead):
    """VERDICT r05 next #4 (missing #4): merge_env.py's module constants reach the kernel
    (bsg_set_params).  Five of them patched -- the HDG action and spawn bearing range, the
    intrusion radius, the waypoint margin, the drift penalty, the intruders' spawn range (so
    intrusions are frequent) -- on the device and, by the same names, on the oracle: every
    output bit-exact / within the bar over 110 steps with NEXT_STEP autoresets, with the
    lookahead (its spawn cache and the lookahead waves' spawns) and without."""
    core, config, nat = bg
    E, N, T = 256, 32, 110
    b = core.DeviceBatch(config.merge_config(num_ac=N, params=PATCHED), E, compute_cd=True,
                         seed=321, lookahead=lookahead)
    o = ob.MergeOracle(E, num_ac=N, seed=321, compute_cd=True, params=PATCHED)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(8)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, N, "merge", t)
    # the patch matters: the unpatched oracle differs
    o2 = ob.MergeOracle(E, num_ac=N, seed=321, compute_cd=True)
    assert not np.array_equal(o2.reset()["obs"], o.reset()["obs"])


def test_merge_env_module_constants_are_live(bg):
    """The drop-in MergeEnv reads merge_env.py's constants at construction, as the reference
    module does: patched D_SPEED / INTRUSION_DISTANCE / SPAWN_DISTANCE_MIN change the env,
    and it matches the oracle restated with the same patch on the same Python-random spawn."""
    import random
    from bluesky_gym.envs import merge_env as me
    from bluesky_gym import spawn as spawnmod
    patch = {"D_SPEED": 35.0, "INTRUSION_DISTANCE": 12.0, "SPAWN_DISTANCE_MIN": 80.0}
    saved = {k: getattr(me, k) for k in patch}
    try:
        for k, v in patch.items():
            setattr(me, k, v)
        env = me.MergeEnv(num_ac=16)
        random.seed(5)
        env.reset()
        random.seed(5)
        sp = spawnmod.merge_spawn(16, spawn_range=(80.0, 200.0))
        o = ob.MergeOracle(1, num_ac=16, autoreset=ob.AUTORESET_NONE, params=patch)
        o.reset(spawn=sp[None, :])
        rng = np.random.default_rng(4)
        for t in range(30):
            a = rng.uniform(-1, 1, 2)
            obs, rew, term, trunc, info = env.step(a)
            r = o.step(a[None, :])
            close(env.batch.obs.cpu().numpy(), r["obs"], f"obs t={t}")
            close([rew], r["reward"], f"reward t={t}")
            assert info["total_intrusions"] == int(o.info()["total_intrusions"][0])
    finally:
        for k, v in saved.items():
            setattr(me, k, v)


@pytest.mark.parametrize("N", [6, 32])
def test_vertical_batch_autoreset_parity(bg, N):
    core, config, nat = bg
    E, T = 128, 100
    b = core.DeviceBatch(config.vertical_config(num_intruders=N - 1), E, compute_cd=True, seed=99)
    o = ob.VerticalOracle(E, num_ac=N, seed=99, compute_cd=True)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(3)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, N, "vertical", t)


@pytest.mark.parametrize("N,autoreset", [(6, ob.AUTORESET_NEXT_STEP), (6, ob.AUTORESET_SAME_STEP),
                                         (32, ob.AUTORESET_NEXT_STEP)])
def test_horizontal_batch_autoreset_parity(bg, N, autoreset):
    """Device Philox spawns, random headings, short TimeLimit (40) so that every env
    auto-resets at least twice; waypoint reaches terminate some episodes early."""
    core, config, nat = bg
    E, T = 128, 90
    b = core.DeviceBatch(config.horizontal_config(num_intruders=N - 1, max_episode_steps=40), E,
                         autoreset=autoreset, compute_cd=True, seed=17)
    o = ob.HorizontalOracle(E, num_ac=N, seed=17, compute_cd=True, max_episode_steps=40,
                            autoreset=autoreset)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(5)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, N, "horizontal", t)
        if autoreset == ob.AUTORESET_SAME_STEP and r["final_obs"] is not None:
            d = r["terminated"] | r["truncated"]
            close(b.final_obs.cpu().numpy()[d], r["final_obs"][d], f"final_obs t={t}")
    # device asin/atan2 vs host libm: the waypoint agrees to a few ulp (~1e-14 deg)
    np.testing.assert_allclose(b.envs["env_wpt_lat"].cpu().numpy(), o.wpt_lat, rtol=0, atol=1e-12)
    np.testing.assert_allclose(b.envs["env_wpt_lon"].cpu().numpy(), o.wpt_lon, rtol=0, atol=1e-12)


def test_descent_batch_autoreset_parity(bg):
    core, config, nat = bg
    E, T = 512, 100
    b = core.DeviceBatch(config.descent_config(), E, seed=5)
    o = ob.DescentOracle(E, seed=5)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(11)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, 1, "descent", t)


def _subset_compare(b, r, ids, N, kind, t, errs):
    """Every output of a strided subset of a full-size device batch vs the subset oracle
    (same global env ids -> same Philox spawns): obs and reward within tolerance,
    terminated / truncated / top-K / intrusion / conflict / LoS bit-exact, tcpamax and
    min_sep within tolerance.  errs accumulates the per-obs-key max |gpu - ref|."""
    o = b.obs.cpu().numpy()[ids]
    close(o, r["obs"], f"obs t={t}")
    for key, (a, z) in errs["slices"].items():
        errs["max"][key] = max(errs["max"].get(key, 0.0),
                               float(np.abs(o[:, a:z].astype(np.float64) - r["obs"][:, a:z]).max()))
        errs.setdefault("ref", {})[key] = max(errs.get("ref", {}).get(key, 0.0),
                                              float(np.abs(r["obs"][:, a:z]).max()))
    rw = b.reward.cpu().numpy()[ids].astype(np.float64)
    close(rw, r["reward"], f"reward t={t}")
    errs["max"]["(reward)"] = max(errs["max"].get("(reward)", 0.0), float(np.abs(rw - r["reward"]).max()))
    assert np.array_equal(b.terminated.cpu().numpy()[ids].astype(bool), r["terminated"]), t
    assert np.array_equal(b.truncated.cpu().numpy()[ids].astype(bool), r["truncated"]), t
    if kind == "descent":
        return
    gi = b.intr_mask.cpu().numpy()[ids].astype(np.uint64)
    assert np.array_equal(gi, r["intr_mask"]), t          # reset steps included (mask 0)
    assert np.array_equal(b.conf_mask.cpu().numpy()[ids].astype(np.uint64), r["conf_mask"]), t
    assert np.array_equal(b.los_mask.cpu().numpy()[ids].astype(np.uint64), r["los_mask"]), t
    close(b.tcpamax.cpu().numpy()[ids], r["tcpamax"], f"tcpamax t={t}", atol=TCPA_ATOL)
    ms_g = b.min_sep.cpu().numpy()[ids].astype(np.float64)
    assert np.array_equal(np.isinf(ms_g), np.isinf(r["min_sep"])), t
    fin = np.isfinite(r["min_sep"])
    close(ms_g[fin], r["min_sep"][fin], f"min_sep t={t}")
    if kind == "merge":
        # reset steps included: the reset observation's top-K (merge_env.py:124, 196)
        assert np.array_equal(b.topk.cpu().numpy()[ids], r["topk"]), t


def _obs_slices(b):
    from bluesky_gym.obs_layout import ObsLayout
    lay = ObsLayout(b.cfg.kind, b.cfg.num_ac, b.cfg.num_ac_state)
    return {k: (sl.start, sl.stop) for k, sl in lay.slices.items()}


def _report(errs, what):
    """Print each obs key's max error and hold the normalised keys (|ref| <= 8, where an fp32
    ulp is <= 1e-6) to north_star's flat 1e-5; raw-unit keys (airspeed in m/s, whose fp32
    ulp is 1.5e-5 at 200 m/s) keep the 1e-5 + 1e-5 |ref| bar of close()."""
    print(f"\n{what}: per-key max |gpu - oracle| over the subset and all compared steps")
    ref = errs.get("ref", {})
    for k, v in sorted(errs["max"].items()):
        print(f"  {k:24s} {v:.3e}   max |ref| {ref.get(k, float('nan')):.3g}")
    flat = {k: v for k, v in errs["max"].items() if k in ref and ref[k] <= 8.0}
    bad = {k: v for k, v in flat.items() if v > 1e-5}
    assert not bad, f"{what}: normalised keys above the flat 1e-5: {bad}"


def test_merge_full_size_subset_parity(bg):
    """BASELINE workload (4096 envs x 32 aircraft): run the full batch on the GPU and
    check a strided subset of 64 envs against the oracle on every output, every step
    (envs are independent, so the subset oracle with the same global env ids sees
    identical spawns)."""
    core, config, nat = bg
    E, N, T = 4096, 32, 60
    b = core.DeviceBatch(config.merge_config(num_ac=N), E, compute_cd=True, seed=42)
    ids = np.arange(0, E, 64)
    o = ob.MergeOracle(len(ids), num_ac=N, seed=42, compute_cd=True)
    o.env_ids = ids
    close(b.reset().cpu().numpy()[ids], o.reset()["obs"], "reset obs")
    errs = {"slices": _obs_slices(b), "max": {}}
    rng = np.random.default_rng(1)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a[ids])
        _subset_compare(b, r, ids, N, "merge", t, errs)
    _report(errs, "merge 4096x32")
    # size-independent properties over the whole batch
    obs = b.obs.cpu().numpy()
    assert np.isfinite(obs).all()
    tk = b.topk.cpu().numpy()
    assert ((tk >= 1) & (tk < N)).all()
    assert all(len(set(row)) == tk.shape[1] for row in tk)
    cm = b.conf_mask.cpu().numpy().astype(np.uint64)
    diag = (cm >> np.arange(N, dtype=np.uint64)[None, :]) & np.uint64(1)
    assert not diag.any()                                  # no self-conflicts
    # StateBased conflicts are symmetric in exact arithmetic; fp rounding may break a
    # near-threshold pair, so only require near-symmetry
    bm = bits(cm, N)
    assert (bm != bm.transpose(0, 2, 1)).sum() <= max(4, bm.sum() // 1000)


def test_descent_full_size_subset_parity(bg):
    """BASELINE configs[4]'s env batch: DescentEnv-v0 x 4096 envs on one GPU (the
    8-GPU run shards the same envs), NEXT_STEP autoreset over 320 steps (every env
    terminates or truncates at least once), a strided 128-env subset vs DescentOracle
    every step, plus whole-batch properties."""
    core, config, nat = bg
    E, T = 4096, 320
    b = core.DeviceBatch(config.descent_config(), E, seed=8)
    ids = np.arange(0, E, 32)
    o = ob.DescentOracle(len(ids), seed=8)
    o.env_ids = ids
    close(b.reset().cpu().numpy()[ids], o.reset()["obs"], "reset obs")
    errs = {"slices": _obs_slices(b), "max": {}}
    rng = np.random.default_rng(21)
    done = np.zeros(E, bool)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        r = o.step(a[ids])
        _subset_compare(b, r, ids, 1, "descent", t, errs)
        done |= (b.terminated | b.truncated).cpu().numpy().astype(bool)
    _report(errs, "descent 4096")
    assert done.all()
    assert np.isfinite(b.obs.cpu().numpy()).all()
    for f, v in b.state.items():
        if v.dtype == torch.float64:
            assert torch.isfinite(v).all(), f


@pytest.mark.parametrize("kind,E,N,T,stride", [
    ("merge", 1024, 16, 60, 16),       # BASELINE.json configs[1]: MergeEnv-v0 1024 envs x 16 aircraft
    ("vertical", 2048, 32, 30, 32),    # configs[2]: VerticalCREnv-v0 2048 envs x 32 aircraft
])
def test_baseline_config_subset_parity(bg, kind, E, N, T, stride):
    """The BASELINE.json parity configs at full size on the GPU: a strided subset of 64
    envs checked against the oracle every step (same global env ids -> same Philox
    spawns), NEXT_STEP autoreset inside the run, plus whole-batch properties."""
    core, config, nat = bg
    if kind == "merge":
        cfg, A = config.merge_config(num_ac=N), 2
        mk = lambda n: ob.MergeOracle(n, num_ac=N, seed=77, compute_cd=True)  # noqa: E731
    else:
        cfg, A = config.vertical_config(num_intruders=N - 1), 1
        mk = lambda n: ob.VerticalOracle(n, num_ac=N, seed=77, compute_cd=True)  # noqa: E731
    b = core.DeviceBatch(cfg, E, compute_cd=True, seed=77)
    ids = np.arange(0, E, stride)
    o = mk(len(ids))
    o.env_ids = ids
    close(b.reset().cpu().numpy()[ids], o.reset()["obs"], "reset obs")
    errs = {"slices": _obs_slices(b), "max": {}}
    rng = np.random.default_rng(9)
    resets = 0
    for t in range(T):
        a = rng.uniform(-1, 1, (E, A))
        b.step(torch.from_numpy(a))
        r = o.step(a[ids])
        # every output, reset steps included; tcpamax / min_sep too
        _subset_compare(b, r, ids, N, kind, t, errs)
        resets += int(r["was_reset"].sum())
    # north_star's flat 1e-5 on the normalised obs keys
    _report(errs, f"{kind} {E}x{N}")
    assert resets > 0 or kind == "vertical"
    obs = b.obs.cpu().numpy()
    assert np.isfinite(obs).all()
    cm = b.conf_mask.cpu().numpy().astype(np.uint64)
    diag = (cm >> np.arange(N, dtype=np.uint64)[None, :]) & np.uint64(1)
    assert not diag.any()


@pytest.mark.parametrize("kind,E,N,K", [
    ("merge", 1, 2, 1),       # one env, the smallest Merge (one intruder, top-1)
    ("merge", 7, 20, 5),      # reference default N = 20 (12 idle lanes of 32), ragged last wave
    ("merge", 5, 5, 4),       # N = 5 -> 8-lane groups, 8 envs per wave, one partial wave
    ("merge", 3, 64, 5),      # maximum aircraft: one env per wave, every lane an aircraft
    ("vertical", 9, 3, 0),    # two intruders, ragged
    ("vertical", 2, 64, 0),   # maximum aircraft (63 intruders)
])
def test_edge_shapes_parity(bg, kind, E, N, K):
    """Ragged batches (E not a multiple of envs per wave), group sizes that leave idle
    lanes, and the minimum/maximum aircraft counts: every output vs the oracle over two
    NEXT_STEP autoresets (short TimeLimit)."""
    core, config, nat = bg
    T, M = 45, 20
    if kind == "merge":
        cfg = config.merge_config(num_ac=N, num_ac_state=K, max_episode_steps=M)
        o = ob.MergeOracle(E, num_ac=N, num_ac_state=K, seed=5, compute_cd=True,
                           max_episode_steps=M)
        A = 2
    else:
        cfg = config.vertical_config(num_intruders=N - 1, max_episode_steps=M)
        o = ob.VerticalOracle(E, num_ac=N, seed=5, compute_cd=True, max_episode_steps=M)
        A = 1
    b = core.DeviceBatch(cfg, E, compute_cd=True, seed=5)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    rng = np.random.default_rng(13)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, A))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare_step(b, r, N, kind, t)


@pytest.mark.parametrize("kind", ["merge", "vertical", "descent", "horizontal", "plan"])
def test_memo_cache_is_bit_exact(bg, kind):
    """The cross-step memo (memo_cache) only skips re-evaluating pure functions of
    unchanged inputs: a batch stepped with it and one stepped without it hold bit-identical
    aircraft state and outputs after every step (climbing/descending aircraft exercise the
    non-level branch, autoresets the invalidation)."""
    core, config, nat = bg
    cfg, E, A = {
        "merge": (config.merge_config(num_ac=32, max_episode_steps=25), 256, 2),
        "vertical": (config.vertical_config(num_intruders=7, max_episode_steps=40), 128, 1),
        "descent": (config.descent_config(max_episode_steps=40), 256, 1),
        "horizontal": (config.horizontal_config(num_intruders=7, max_episode_steps=30), 128, 1),
        "plan": (config.plan_waypoint_config(max_episode_steps=30), 256, 1),
    }[kind]
    with_m = core.DeviceBatch(cfg, E, compute_cd=True, seed=21, memo_cache=True)
    no_m = core.DeviceBatch(cfg, E, compute_cd=True, seed=21, memo_cache=False)
    with_m.reset()
    no_m.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4)
    for t in range(70):
        a = torch.rand((E, A), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
        o1, r1, te1, tr1 = with_m.step(a)
        o2, r2, te2, tr2 = no_m.step(a)
        assert torch.equal(o1, o2) and torch.equal(r1, r2), t
        assert torch.equal(te1, te2) and torch.equal(tr1, tr2), t
        for f, v in with_m.state.items():
            assert torch.equal(v.view(torch.int64) if v.dtype == torch.float64 else v,
                               no_m.state[f].view(torch.int64) if v.dtype == torch.float64
                               else no_m.state[f]), (t, f)


def test_merge_full_size_soak_300_steps(bg):
    """The bench workload for 300 RL steps (six TimeLimit episodes per env, thousands of
    autoresets): a strided 32-env subset stays on the oracle every 10th step (outputs and
    masks), and the whole batch keeps finite state, valid top-K and in-range counters."""
    core, config, nat = bg
    E, N, T = 4096, 32, 300
    b = core.DeviceBatch(config.merge_config(num_ac=N), E, compute_cd=True, seed=2024)
    ids = np.arange(0, E, 128)
    o = ob.MergeOracle(len(ids), num_ac=N, seed=2024, compute_cd=True)
    o.env_ids = ids
    b.reset()
    o.reset()
    errs = {"slices": _obs_slices(b), "max": {}}
    rng = np.random.default_rng(77)
    for t in range(T):
        a = rng.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a[ids])
        if t % 10 == 9:
            _subset_compare(b, r, ids, N, "merge", t, errs)
    for f, v in b.state.items():
        if v.dtype == torch.float64:
            assert torch.isfinite(v).all(), f
    _report(errs, "merge 4096x32, 300-step soak")
    sc = b.envs["step_count"].cpu().numpy()
    assert sc.min() >= 0 and sc.max() <= 50
    tk = b.topk.cpu().numpy()
    assert ((tk >= 1) & (tk < N)).all()
    assert np.isfinite(b.obs.cpu().numpy()).all()
