"""GPU parity of StaticObstacleEnv-v0 and SectorCREnv-v0 (polygon
containment, sector_cr_env.py:134-139 / static_obstacle_env.py:329-338).

* golden: the reference env episodes (tests/golden/static.npz, sector_N32.npz) replayed
  through the HIP kernel from the recorded host spawn rows -- geometry, obs, rewards,
  terminations / truncations (sector exit) and intrusion masks;
* batch: device Philox resets (polygon generation, rejection sampling, waypoint
  rank-assignment on the device) against the CPU oracle's restatement of the same draws,
  with autoreset in both modes and StateBased CD over the variable aircraft count.
"""
import numpy as np
import pytest
import torch

import oracle_replay as rp
from oracle import areas as oa
from oracle import batched as ob
from oracle import batched_areas as oba
from test_gpu_parity import TCPA_ATOL, bits, close, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bg():
    from bluesky_gym import config, core, _native
    return core, config, _native


def test_static_golden_on_gpu(bg):
    core, config, nat = bg
    g = load("static")
    n_ep, T = g["actions"].shape[:2]
    b = core.DeviceBatch(config.static_config(), n_ep, autoreset=nat.AUTORESET_NONE)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    geo = b.envs["env_geom"].cpu().numpy()
    W = 6 + 2 * oa.STATIC_VMAX
    np.testing.assert_allclose(geo[:, 0:2], g["wpt"], rtol=0, atol=1e-12)
    for o in range(oa.STATIC_NUM_OBSTACLES):
        h = geo[:, 2 + o * W: 2 + (o + 1) * W]
        np.testing.assert_allclose(h[:, 0], g["clat"][:, o], rtol=0, atol=1e-12)
        np.testing.assert_allclose(h[:, 1], g["clon"][:, o], rtol=0, atol=1e-12)
        np.testing.assert_allclose(h[:, 2], g["R"][:, o], rtol=1e-15, atol=0)
        assert np.array_equal(h[:, 3].astype(int), g["nvert"][:, o])
        for e in range(n_ep):
            n = int(g["nvert"][e, o])
            np.testing.assert_allclose(h[e, 6:6 + n], g["poly_lat"][e, o, :n], rtol=0, atol=1e-12)
            np.testing.assert_allclose(h[e, 6 + oa.STATIC_VMAX:6 + oa.STATIC_VMAX + n],
                                       g["poly_lon"][e, o, :n], rtol=0, atol=1e-12)
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


def test_sector_golden_on_gpu(bg):
    core, config, nat = bg
    g = load("sector_N32")
    n_ep, T = g["actions"].shape[:2]
    N = int(g["num_ac"])
    b = core.DeviceBatch(config.sector_config(num_ac=N), n_ep, autoreset=nat.AUTORESET_NONE,
                         compute_cd=True)
    obs0 = b.reset(spawn=torch.from_numpy(g["spawn"])).cpu().numpy()
    close(obs0, g["obs0"], "reset obs")
    assert np.array_equal(b.envs["env_geom"].cpu().numpy()[:, 0].astype(int), g["num_ac_ep"])
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
        ib = bits(b.intr_mask.cpu().numpy(), N)[:, 1:]
        assert np.array_equal(ib[live], g["intr"][live, t]), t


def _cmp(b, r, t, cd):
    close(b.obs.cpu().numpy(), r["obs"], f"obs t={t}")
    close(b.reward.cpu().numpy(), r["reward"], f"reward t={t}")
    assert np.array_equal(b.terminated.cpu().numpy().astype(bool), r["terminated"]), t
    assert np.array_equal(b.truncated.cpu().numpy().astype(bool), r["truncated"]), t
    if cd:
        # reset steps included (no intrusion check at a reset: mask 0)
        assert np.array_equal(b.intr_mask.cpu().numpy().astype(np.uint64), r["intr_mask"]), t
        assert np.array_equal(b.conf_mask.cpu().numpy().astype(np.uint64), r["conf_mask"]), t
        assert np.array_equal(b.los_mask.cpu().numpy().astype(np.uint64), r["los_mask"]), t
        close(b.tcpamax.cpu().numpy(), r["tcpamax"], f"tcpamax t={t}", atol=TCPA_ATOL)
        ms_g = b.min_sep.cpu().numpy().astype(np.float64)
        assert np.array_equal(np.isinf(ms_g), np.isinf(r["min_sep"])), t
        fin = np.isfinite(r["min_sep"])
        close(ms_g[fin], r["min_sep"][fin], f"min_sep t={t}")


@pytest.mark.parametrize("autoreset", [ob.AUTORESET_NEXT_STEP, ob.AUTORESET_SAME_STEP])
def test_static_batch_autoreset_parity(bg, autoreset):
    core, config, nat = bg
    E, T = 48, 45
    b = core.DeviceBatch(config.static_config(max_episode_steps=20), E, autoreset=autoreset, seed=21)
    o = oba.StaticOracle(E, max_episode_steps=20, autoreset=autoreset, seed=21)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    ra = np.random.default_rng(4)
    for t in range(T):
        a = ra.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _cmp(b, r, t, cd=False)
        if autoreset == ob.AUTORESET_SAME_STEP and r["final_obs"] is not None:
            d = r["terminated"] | r["truncated"]
            close(b.final_obs.cpu().numpy()[d], r["final_obs"][d], f"final_obs t={t}")


@pytest.mark.parametrize("autoreset,mode", [(ob.AUTORESET_NEXT_STEP, "normal"),
                                            (ob.AUTORESET_SAME_STEP, "uniform")])
def test_sector_batch_autoreset_parity(bg, autoreset, mode):
    core, config, nat = bg
    E, N, T = 32, 32, 50
    b = core.DeviceBatch(config.sector_config(num_ac=N, max_episode_steps=20, density_mode=mode),
                         E, autoreset=autoreset, compute_cd=True, seed=33)
    o = oba.SectorOracle(E, num_ac=N, max_episode_steps=20, autoreset=autoreset, seed=33,
                         compute_cd=True, density_mode=mode)
    close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
    assert np.array_equal(b.envs["env_geom"].cpu().numpy()[:, 0].astype(int), o.nac)
    ra = np.random.default_rng(6)
    for t in range(T):
        a = ra.uniform(-1, 1, (E, 2))
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _cmp(b, r, t, cd=True)
        assert np.array_equal(b.envs["env_geom"].cpu().numpy()[:, 0].astype(int), o.nac), t
        if autoreset == ob.AUTORESET_SAME_STEP and r["final_obs"] is not None:
            d = r["terminated"] | r["truncated"]
            close(b.final_obs.cpu().numpy()[d], r["final_obs"][d], f"final_obs t={t}")


def test_gym_make_static_and_sector_reproduce_reference():
    import bluesky_gym
    from bluesky_gym import _gym
    bluesky_gym.register_envs()
    for name, eid in (("static", "StaticObstacleEnv-v0"), ("sector_N32", "SectorCREnv-v0")):
        g = load(name)
        np.random.seed(int(g["seed"]))
        env = _gym.make(eid)
        keys = sorted(env.observation_space.spaces)
        for ep in range(len(g["length"])):
            obs, _ = env.reset()
            close(np.concatenate([obs[k] for k in keys]), g["obs0"][ep], f"{name} reset {ep}")
            for t in range(g["length"][ep]):
                obs, rew, term, trunc, info = env.step(g["actions"][ep, t])
                close(np.concatenate([obs[k] for k in keys]), g["obs"][ep, t], f"{name} {ep},{t}")
                close(rew, g["reward"][ep, t], f"{name} reward {ep},{t}")
                assert int(term) == g["terminated"][ep, t]
                assert bool(trunc) == bool(g["truncated"][ep, t])
        env.close()
