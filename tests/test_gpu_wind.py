"""GPU parity of the wind path (bluesky_gym/wrappers/wind.py).

* golden: the reference WindFieldWrapper(augment_obs=True) around each reference env,
  recorded by tests/golden/make_golden.py, replayed through the HIP kernel;
* batch: device Philox spawns + random actions, every output (incl. StateBased CD on the
  wind-affected ground speed / track) against the CPU oracle, for a 2-D field, a field of
  more points than the kernel keeps in registers, and altitude profiles;
* API: WindFieldWrapper / NoisyObservationWrapper on gym.make envs reproduce the
  reference episodes.

Tolerances as in test_gpu_parity.py (obs / rewards 1e-5 abs + 1e-5 rel).  The wind path
adds asin/atan2 of the wind triangle, whose device results may differ from glibc's in
the last ulp, so the state is compared with a tolerance here rather than bit for bit.
"""
import numpy as np
import pytest
import torch

import oracle_replay as rp
from oracle import batched as ob
from oracle import bluesky_subset as bsx
from test_gpu_parity import ATOL, RTOL, TCPA_ATOL, bits, close, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bg():
    from bluesky_gym import config, core, _native
    from bluesky_gym.wind import WindTable
    return core, config, _native, WindTable


def _table(WindTable, g):
    return WindTable(g["wind_lat"], g["wind_lon"], g["wind_vnorth"], g["wind_veast"],
                     g["wind_alt"] if "wind_alt" in g else None)


def _kind_cfg(config, kind, N):
    return {"merge": lambda: config.merge_config(num_ac=N),
            "vertical": lambda: config.vertical_config(num_intruders=N - 1),
            "descent": lambda: config.descent_config(),
            "horizontal": lambda: config.horizontal_config(num_intruders=N - 1)}[kind]()


@pytest.mark.parametrize("name", ["wind_merge_N16", "wind_vertical_N6", "wind_descent",
                                  "wind_horizontal_N6"])
def test_wind_golden_on_gpu(bg, name):
    core, config, nat, WindTable = bg
    g = load(name)
    kind = name.split("_")[1]
    n_ep, T = g["actions"].shape[:2]
    N = int(g["num_ac"]) if "num_ac" in g else 1
    b = core.DeviceBatch(_kind_cfg(config, kind, N), n_ep, autoreset=nat.AUTORESET_NONE,
                         compute_cd=kind != "descent")
    b.set_wind(_table(WindTable, g), augment_obs=True)
    assert b.obs_dim == g["obs"].shape[-1]
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    m = rp.step_mask(g)
    act = torch.from_numpy(g["actions"]).cuda()
    for t in range(T):
        obs, rew, term, trunc = b.step(act[:, t])
        live = m[:, t]
        if not live.any():
            break
        go = g["obs"][live, t]
        fin = np.isfinite(go)          # NaN wind keys: the reference wrapper raised there
        close(obs.cpu().numpy()[live][fin], go[fin], f"obs t={t}")
        close(rew.cpu().numpy()[live], g["reward"][live, t], f"reward t={t}")
        assert np.array_equal(term.cpu().numpy()[live], g["terminated"][live, t].astype(np.uint8)), t


def _compare(b, r, N, t, state_tol=True, o=None):
    close(b.obs.cpu().numpy(), r["obs"], f"obs t={t}")
    close(b.reward.cpu().numpy(), r["reward"], f"reward t={t}")
    assert np.array_equal(b.terminated.cpu().numpy().astype(bool), r["terminated"]), t
    assert np.array_equal(b.truncated.cpu().numpy().astype(bool), r["truncated"]), t
    if "conf_mask" in r:
        assert np.array_equal(b.conf_mask.cpu().numpy().astype(np.uint64), r["conf_mask"]), t
        assert np.array_equal(b.los_mask.cpu().numpy().astype(np.uint64), r["los_mask"]), t
        close(b.tcpamax.cpu().numpy(), r["tcpamax"], f"tcpamax t={t}", atol=TCPA_ATOL)
    if o is not None:
        for f in ("lat", "lon"):
            close(b.state[f].cpu().numpy(), getattr(o.st, f), f"{f} t={t}", atol=1e-9)
        for f in ("hdg", "trk"):
            d = np.abs(b.state[f].cpu().numpy() - getattr(o.st, f))
            d = np.minimum(d, 360.0 - d)
            assert d.max() <= 1e-7, (f, t, d.max())
        close(b.state["gs"].cpu().numpy(), o.st.gs, f"gs t={t}", atol=1e-8)


def _merge_field(P, rng):
    lat = rng.uniform(52.3, 54.3, P)
    lon = rng.uniform(3.8, 5.6, P)
    return lat, lon, rng.uniform(-20, 20, (1, P)), rng.uniform(-20, 20, (1, P))


@pytest.mark.parametrize("P,autoreset", [(4, ob.AUTORESET_NEXT_STEP), (12, ob.AUTORESET_SAME_STEP),
                                         (1, ob.AUTORESET_NEXT_STEP)])
def test_merge_wind_batch_parity(bg, P, autoreset):
    core, config, nat, WindTable = bg
    E, N, T = 128, 32, 60
    rng = np.random.default_rng(P)
    lat, lon, vn, ve = _merge_field(P, rng)
    b = core.DeviceBatch(config.merge_config(num_ac=N), E, autoreset=autoreset, compute_cd=True,
                         seed=77)
    b.set_wind(WindTable(lat, lon, vn, ve), augment_obs=True)
    o = ob.MergeOracle(E, num_ac=N, autoreset=autoreset, seed=77, compute_cd=True)
    f = bsx.WindField()
    f.addpointvne(lat, lon, vn, ve)
    o.set_wind(f, augment_obs=True)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    ra = np.random.default_rng(3)
    for t in range(T):
        a = ra.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare(b, r, N, t, o=o)


def test_vertical_wind_profiles_batch_parity(bg):
    core, config, nat, WindTable = bg
    E, N, T = 128, 8, 80
    lat = np.array([51.9, 51.9, 52.1, 52.1, 52.0])
    lon = np.array([3.9, 4.1, 3.9, 4.1, 4.0])
    alt = np.array([0.0, 1500.0, 3000.0, 6000.0])
    rng = np.random.default_rng(5)
    vn, ve = rng.uniform(-25, 25, (4, 5)), rng.uniform(-25, 25, (4, 5))
    b = core.DeviceBatch(config.vertical_config(num_intruders=N - 1), E, compute_cd=True, seed=8)
    b.set_wind(WindTable(lat, lon, vn, ve, alt), augment_obs=True)
    o = ob.VerticalOracle(E, num_ac=N, seed=8, compute_cd=True)
    f = bsx.WindField()
    f.addpointvne(lat, lon, vn, ve, alt)
    o.set_wind(f, augment_obs=True)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    ra = np.random.default_rng(9)
    for t in range(T):
        a = ra.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _compare(b, r, N, t, o=o)


def test_wind_wrappers_on_gym_make_reproduce_reference():
    import bluesky_gym
    from bluesky_gym import _gym
    from bluesky_gym.envs import merge_env as me
    from bluesky_gym.wrappers import NoisyObservationWrapper, WindFieldWrapper
    import random
    bluesky_gym.register_envs()
    # wind: the reference WindFieldWrapper episodes (augment_obs=True)
    g = load("wind_merge_N16")
    me.NUM_AC = int(g["num_ac"])
    try:
        random.seed(int(g["seed"]))
        env = WindFieldWrapper(_gym.make("MergeEnv-v0"), lat=g["wind_lat"], lon=g["wind_lon"],
                               vnorth=g["wind_vnorth"], veast=g["wind_veast"], augment_obs=True)
        keys = sorted(env.observation_space.spaces)
        assert "wind_u" in keys and len(keys) == 14
        for ep in range(len(g["length"])):
            obs, _ = env.reset()
            close(np.concatenate([obs[k] for k in keys]), g["obs0"][ep], f"reset {ep}")
            for t in range(g["length"][ep]):
                obs, rew, term, trunc, info = env.step(g["actions"][ep, t])
                close(np.concatenate([obs[k] for k in keys]), g["obs"][ep, t], f"obs {ep},{t}")
                close(rew, g["reward"][ep, t], f"reward {ep},{t}")
        env.close()
        # noise: the reference NoisyObservationWrapper episodes
        g = load("noisy_merge_N8")
        me.NUM_AC = int(g["num_ac"])
        random.seed(int(g["seed"]))
        np.random.seed(int(g["seed"]) + 1000)
        env = NoisyObservationWrapper(_gym.make("MergeEnv-v0"), noise_level=float(g["noise"]))
        keys = sorted(env.observation_space.spaces)
        for ep in range(len(g["length"])):
            obs, _ = env.reset()
            close(np.concatenate([obs[k] for k in keys]), g["obs0"][ep], f"noisy reset {ep}")
            for t in range(g["length"][ep]):
                obs, *_ = env.step(g["actions"][ep, t])
                close(np.concatenate([obs[k] for k in keys]), g["obs"][ep, t], f"noisy {ep},{t}")
        env.close()
    finally:
        me.NUM_AC = 20


def test_make_vec_with_wind_wrapper():
    import bluesky_gym
    from bluesky_gym import _gym
    from bluesky_gym.wrappers import VectorWindFieldWrapper
    bluesky_gym.register_envs()
    venv = _gym.make_vec("VerticalCREnv-v0", num_envs=256, vectorization_mode="vector_entry_point",
                         num_ac=8, seed=3)
    w = VectorWindFieldWrapper(venv, lat=[51.9, 51.9, 52.1, 52.1], lon=[3.9, 4.1, 3.9, 4.1],
                         vnorth=[[16, 12, 14, 15]], veast=[[3, 7, 9, 4]], augment_obs=True)
    obs, _ = w.reset()
    assert obs["wind_u"].shape == (256, 1) and np.all(np.isfinite(obs["wind_u"]))
    assert np.abs(obs["wind_u"]).max() > 0.05
    for _ in range(5):
        obs, rew, term, trunc, info = w.step(np.random.default_rng(0).uniform(-1, 1, (256, 1)))
    assert np.all(np.isfinite(obs["wind_v"]))
    w.close()
