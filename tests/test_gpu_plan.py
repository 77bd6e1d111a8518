"""GPU parity of PlanWaypointEnv-v0 (plan_waypoint_env.py) and of the reset that keeps a
truncated episode's aircraft (Descent / PlanWaypoint: reset() does not clear the traffic,
descent_env.py:173 / plan_waypoint_env.py:164 cre refused; the terminal step deletes the
aircraft, :201-204 / :189-193).

* golden: one env driven over consecutive reference episodes (tests/golden/plan*.npz,
  descent_keep.npz, make_golden.py gen_plan / keep_traffic) replayed through the HIP
  kernel: reset from each spawn row -- keeping the aircraft after a truncation -- then
  the recorded actions; obs, rewards, terminated / truncated, waypoints;
* batch: device Philox resets against the CPU oracle in both autoreset modes, with a
  waypoint-seeking policy so that episodes end by termination (all five reached, aircraft
  re-created) and by truncation (aircraft kept) in the same run.

Tolerances as in test_gpu_parity.py (obs / rewards 1e-5 abs + 1e-5 rel).
"""
import numpy as np
import pytest
import torch

from oracle import batched as ob
from oracle import bluesky_subset as bsx
from test_gpu_parity import close, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bg():
    from bluesky_gym import config, core, _native
    return core, config, _native


def _replay_sequential(b, g):
    """The golden's episodes one after the other through an E=1 batch."""
    n_ep = len(g["length"])
    for ep in range(n_ep):
        obs0 = b.reset(spawn=torch.from_numpy(g["spawn"][ep:ep + 1])).cpu().numpy()[0]
        close(obs0, g["obs0"][ep], f"reset obs ep={ep}")
        if "wpt" in g:
            np.testing.assert_allclose(b.envs["env_geom"].cpu().numpy()[0], g["wpt"][ep],
                                       rtol=0, atol=1e-12)
        for t in range(int(g["length"][ep])):
            obs, rew, term, trunc = b.step(torch.from_numpy(g["actions"][ep, t][None]))
            close(obs.cpu().numpy()[0], g["obs"][ep, t], f"obs ep={ep} t={t}")
            close(rew.cpu().numpy()[0], g["reward"][ep, t], f"reward ep={ep} t={t}")
            assert int(term.cpu()[0]) == g["terminated"][ep, t], (ep, t)
            assert int(trunc.cpu()[0]) == g["truncated"][ep, t], (ep, t)
            if not g["terminated"][ep, t]:
                st = np.array([b.state[k].cpu().numpy()[0, 0] for k in
                               ("lat", "lon", "alt", "hdg", "tas", "cas", "vs")])
                np.testing.assert_allclose(st, g["state"][ep, t][:, 0], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("name", ["plan", "plan_long", "plan_greedy"])
def test_plan_golden_sequential_on_gpu(bg, name):
    core, config, nat = bg
    g = load(name)
    T = g["actions"].shape[1]
    b = core.DeviceBatch(config.plan_waypoint_config(max_episode_steps=T), 1,
                         autoreset=nat.AUTORESET_NONE)
    _replay_sequential(b, g)


def test_descent_keep_golden_sequential_on_gpu(bg):
    core, config, nat = bg
    g = load("descent_keep")
    T = g["actions"].shape[1]
    b = core.DeviceBatch(config.descent_config(max_episode_steps=T), 1,
                         autoreset=nat.AUTORESET_NONE)
    _replay_sequential(b, g)


def _seek(obs_flat):
    """Steer at the nearest unreached waypoint (same policy for oracle and device)."""
    W = 5
    cos_d, sin_d = obs_flat[:, 0:W], obs_flat[:, W:2 * W]
    dist, reached = obs_flat[:, 2 * W:3 * W], obs_flat[:, 3 * W:4 * W]
    d = np.where(reached == 0, dist, np.inf)
    k = np.argmin(d, axis=1)
    rows = np.arange(len(k))
    drift = np.degrees(np.arctan2(sin_d[rows, k], cos_d[rows, k]))
    return np.clip(-drift / 45.0, -1.0, 1.0)[:, None]


def _degenerate(dev, ref):
    """A waypoint drawn at distance 0 (randint(0, 75) includes 0) sits on the aircraft:
    its bearing -- hence cos/sin_difference in the reset observation -- is atan2 of
    rounding noise (|d| ~ 1e-14 NM) in the reference and here alike.  Those two terms
    are checked for being a unit vector only; everything else is compared as usual."""
    dev = dev.copy()
    W = 5
    deg = ref[:, 2 * W:3 * W] < 1e-9
    deg &= ref[:, 3 * W:4 * W] == 0
    if deg.any():
        c, s_ = dev[:, 0:W], dev[:, W:2 * W]
        np.testing.assert_allclose((c * c + s_ * s_)[deg], 1.0, atol=1e-5)
        dev[:, 0:W][deg] = ref[:, 0:W][deg]
        dev[:, W:2 * W][deg] = ref[:, W:2 * W][deg]
    return dev


def _cmp(b, r, t):
    close(_degenerate(b.obs.cpu().numpy(), r["obs"]), r["obs"], f"obs t={t}")
    close(b.reward.cpu().numpy(), r["reward"], f"reward t={t}")
    assert np.array_equal(b.terminated.cpu().numpy().astype(bool), r["terminated"]), t
    assert np.array_equal(b.truncated.cpu().numpy().astype(bool), r["truncated"]), t


@pytest.mark.parametrize("autoreset", [ob.AUTORESET_NEXT_STEP, ob.AUTORESET_SAME_STEP])
def test_plan_batch_autoreset_parity(bg, autoreset):
    core, config, nat = bg
    E, T, L = 256, 240, 90
    b = core.DeviceBatch(config.plan_waypoint_config(max_episode_steps=L), E,
                         autoreset=autoreset, seed=41)
    o = ob.PlanWaypointOracle(E, max_episode_steps=L, autoreset=autoreset, seed=41)
    r = o.reset()
    close(_degenerate(b.reset().cpu().numpy(), r["obs"]), r["obs"], "reset obs")
    np.testing.assert_allclose(b.envs["env_geom"].cpu().numpy(),
                               np.concatenate([o.wpt_lat, o.wpt_lon], 1), rtol=0, atol=1e-12)
    obs = r["obs"]
    n_term = n_trunc = 0
    for t in range(T):
        a = _seek(obs)
        b.step(torch.from_numpy(a))
        r = o.step(a)
        _cmp(b, r, t)
        if autoreset == ob.AUTORESET_SAME_STEP and r["final_obs"] is not None:
            d = r["terminated"] | r["truncated"]
            close(_degenerate(b.final_obs.cpu().numpy()[d], r["final_obs"][d]), r["final_obs"][d],
                  f"final_obs t={t}")
        fl = b.envs["flags"].cpu().numpy()
        assert np.array_equal((fl & nat.FLAG_AC_PRESENT) != 0, o.present), t
        n_term += int(r["terminated"].sum())
        n_trunc += int(r["truncated"].sum())
        obs = r["obs"]
    assert n_term > 0 and n_trunc > 0, (n_term, n_trunc)
    np.testing.assert_allclose(b.envs["env_geom"].cpu().numpy(),
                               np.concatenate([o.wpt_lat, o.wpt_lon], 1), rtol=0, atol=1e-12)


def test_plan_wind_obs_batch_parity(bg):
    """WindFieldWrapper(augment_obs=True) on PlanWaypoint: wind_u / wind_v sort after
    waypoint_reached (the aircraft fly at 0 ft, below the 50 ft wind floor)."""
    core, config, nat = bg
    from bluesky_gym.wind import WindTable
    E, T = 64, 30
    lat = np.array([51.8, 52.2, 52.0])
    lon = np.array([3.8, 4.0, 4.3])
    rng = np.random.default_rng(2)
    vn, ve = rng.uniform(-20, 20, (1, 3)), rng.uniform(-20, 20, (1, 3))
    b = core.DeviceBatch(config.plan_waypoint_config(max_episode_steps=12), E, seed=3)
    b.set_wind(WindTable(lat, lon, vn, ve), augment_obs=True)
    o = ob.PlanWaypointOracle(E, max_episode_steps=12, seed=3)
    f = bsx.WindField()
    f.addpointvne(lat, lon, vn, ve)
    o.set_wind(f, augment_obs=True)
    r = o.reset()
    close(_degenerate(b.reset().cpu().numpy(), r["obs"]), r["obs"], "reset obs")
    ra = np.random.default_rng(4)
    for t in range(T):
        a = ra.uniform(-1, 1, (E, 1))
        b.step(torch.from_numpy(a))
        _cmp(b, o.step(a), t)


def test_descent_batch_truncation_keeps_aircraft(bg):
    """Descent with a short TimeLimit: truncated envs continue with their aircraft (new
    target altitude drawn), crashed / landed ones start over."""
    core, config, nat = bg
    E, T, L = 256, 60, 6
    for autoreset in (ob.AUTORESET_NEXT_STEP, ob.AUTORESET_SAME_STEP):
        b = core.DeviceBatch(config.descent_config(max_episode_steps=L), E, seed=9,
                             autoreset=autoreset)
        o = ob.DescentOracle(E, max_episode_steps=L, seed=9, autoreset=autoreset)
        close(b.reset().cpu().numpy(), o.reset()["obs"], "reset obs")
        ra = np.random.default_rng(5)
        n_trunc = 0
        for t in range(T):
            a = ra.uniform(-1, 1, (E, 1))
            b.step(torch.from_numpy(a))
            r = o.step(a)
            _cmp(b, r, t)
            n_trunc += int(r["truncated"].sum())
            fl = b.envs["flags"].cpu().numpy()
            assert np.array_equal((fl & nat.FLAG_AC_PRESENT) != 0, o.present), t
        assert n_trunc > 0


def test_gym_make_plan_reproduces_reference():
    import bluesky_gym
    from bluesky_gym import _gym
    bluesky_gym.register_envs()
    g = load("plan_greedy")
    np.random.seed(int(g["seed"]))
    env = _gym.make("PlanWaypointEnv-v0")
    keys = sorted(env.observation_space.spaces)
    for ep in range(len(g["length"])):
        obs, info = env.reset()
        close(np.concatenate([obs[k] for k in keys]), g["obs0"][ep], f"reset {ep}")
        for t in range(g["length"][ep]):
            obs, rew, term, trunc, info = env.step(g["actions"][ep, t])
            close(np.concatenate([obs[k] for k in keys]), g["obs"][ep, t], f"{ep},{t}")
            close(rew, g["reward"][ep, t], f"reward {ep},{t}")
            assert int(term) == g["terminated"][ep, t]
            assert info["waypoints_completed"] == g["info"][ep, t, 1]
        # TimeLimit(300) never fires within the golden's 120 steps: the next reset() after
        # a golden truncation keeps the aircraft exactly like the reference env did
    env.close()


def test_make_vec_plan_waypoint():
    import bluesky_gym
    from bluesky_gym import _gym
    bluesky_gym.register_envs()
    env = _gym.make_vec("PlanWaypointEnv-v0", num_envs=8, vectorization_mode="vector_entry_point")
    obs, info = env.reset()
    assert set(obs) == {"cos_difference", "sin_difference", "waypoint_distance", "waypoint_reached"}
    assert obs["waypoint_distance"].shape == (8, 5)
    obs, rew, term, trunc, info = env.step(np.zeros((8, 1)))
    assert rew.shape == (8,) and "waypoints_completed" in info
    env.close()
