"""Host-side API checks (no GPU): env registry, observation layouts, and that the host
spawn draws consume Python `random` / legacy `np.random` exactly as the reference env
code does (checked against the golden fixtures recorded from the reference)."""
import os
import random

import numpy as np
import pytest

import bluesky_gym
from bluesky_gym import _gym, spawn
from bluesky_gym import _native as nat
from bluesky_gym.obs_layout import ObsLayout
from oracle import batched as ob

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_register_envs_matches_reference_ids_and_limits():
    bluesky_gym.register_envs()
    expect = {"DescentEnv-v0": 300, "PlanWaypointEnv-v0": 300, "HorizontalCREnv-v0": 300,
              "VerticalCREnv-v0": 300, "SectorCREnv-v0": 200, "StaticObstacleEnv-v0": 100,
              "MergeEnv-v0": 50}
    reg = _gym.registry
    for k, v in expect.items():
        assert reg[k].max_episode_steps == v
        assert reg[k].entry_point.startswith("bluesky_gym.envs.")
    for k in expect:
        assert reg[k].vector_entry_point.startswith("bluesky_gym.vector:")
    # no HIP device here: every env id fails loudly instead of falling back to the CPU
    with pytest.raises(nat.BsgError):
        _gym.make("PlanWaypointEnv-v0")


def test_obs_layout_keys_sorted_like_gymnasium():
    m = ObsLayout(nat.ENV_MERGE, 20, 5)
    assert list(m.keys) == list(ob.MERGE_OBS_KEYS) and m.dim == 40
    v = ObsLayout(nat.ENV_VERTICAL_CR, 6, 0)
    assert list(v.keys) == list(ob.VERTICAL_OBS_KEYS) and v.dim == 39
    d = ObsLayout(nat.ENV_DESCENT, 1, 0)
    assert list(d.keys) == list(ob.DESCENT_OBS_KEYS) and d.dim == 4
    h = ObsLayout(nat.ENV_HORIZONTAL_CR, 6, 0)
    assert list(h.keys) == list(ob.HORIZONTAL_OBS_KEYS) and h.dim == 28
    from oracle import batched_areas as oba
    so = ObsLayout(nat.ENV_STATIC_OBSTACLE, 1, 0)
    assert list(so.keys) == list(oba.STATIC_OBS_KEYS) and so.dim == 43
    sc = ObsLayout(nat.ENV_SECTOR_CR, 32, 4)
    assert list(sc.keys) == list(oba.SECTOR_OBS_KEYS) and sc.dim == 31
    pw = ObsLayout(nat.ENV_PLAN_WAYPOINT, 1, 0)
    assert list(pw.keys) == list(ob.PLAN_OBS_KEYS) and pw.dim == 20
    assert pw.bounds["waypoint_reached"] == (0, 1)
    w = ObsLayout(nat.ENV_MERGE, 20, 5, wind=True)
    assert w.dim == 42 and w.slices["wind_u"] == slice(30, 31)
    space = m.observation_space(_gym.spaces)
    assert list(space.spaces) == sorted(space.spaces)


@pytest.mark.parametrize("name,seed", [("merge_N8", 0), ("merge_N16", 1), ("merge_N32", 3)])
def test_merge_host_spawn_consumes_random_like_reference(name, seed):
    g = dict(np.load(f"{GOLD}/{name}.npz"))
    random.seed(seed)
    for ep in range(len(g["length"])):
        assert np.array_equal(spawn.merge_spawn(int(g["num_ac"])), g["spawn"][ep])


@pytest.mark.parametrize("name,seed", [("vertical_N6", 4), ("vertical_N32", 5)])
def test_vertical_host_spawn_consumes_np_random_like_reference(name, seed):
    g = dict(np.load(f"{GOLD}/{name}.npz"))
    np.random.seed(seed)
    for ep in range(len(g["length"])):
        assert np.array_equal(spawn.vertical_spawn(int(g["num_ac"]) - 1), g["spawn"][ep])


def test_descent_host_spawn_consumes_np_random_like_reference():
    g = dict(np.load(f"{GOLD}/descent.npz"))
    np.random.seed(6)
    for ep in range(len(g["length"])):
        assert np.array_equal(spawn.descent_spawn(), g["spawn"][ep])


@pytest.mark.parametrize("name,seed", [("horizontal_N6", 7), ("horizontal_N16", 8)])
def test_horizontal_host_spawn_consumes_np_random_like_reference(name, seed):
    g = dict(np.load(f"{GOLD}/{name}.npz"))
    np.random.seed(seed)
    for ep in range(len(g["length"])):
        assert np.array_equal(spawn.horizontal_spawn(int(g["num_ac"]) - 1), g["spawn"][ep])


def test_device_spawn_draws_in_reference_ranges():
    """The Philox spawn distributions stay inside the reference's randint ranges."""
    o = ob.HorizontalOracle(512, num_ac=6, seed=3)
    sp = o.device_spawn_params(np.arange(512), np.zeros(512))
    dpsi, cpa, tlosh = sp[:, 0:15:3], sp[:, 1:15:3], sp[:, 2:15:3]
    assert dpsi.min() >= 45 and dpsi.max() < 315
    assert cpa.min() >= 0 and cpa.max() < 5
    assert tlosh.min() >= 100 and tlosh.max() < 1000
    assert sp[:, -1].min() >= 100 and sp[:, -1].max() < 150
    assert np.array_equal(sp, np.floor(sp))


def test_static_host_spawn_consumes_np_random_like_reference():
    from bluesky_gym import areas
    g = dict(np.load(f"{GOLD}/static.npz"))
    np.random.seed(int(g["seed"]))
    for ep in range(len(g["length"])):
        assert np.array_equal(areas.static_spawn(), g["spawn"][ep])


def test_sector_host_spawn_consumes_np_random_like_reference():
    from bluesky_gym import areas
    g = dict(np.load(f"{GOLD}/sector_N32.npz"))
    np.random.seed(int(g["seed"]))
    for ep in range(len(g["length"])):
        assert np.array_equal(areas.sector_spawn(int(g["num_ac"])), g["spawn"][ep])


@pytest.mark.parametrize("name", ["plan", "plan_greedy"])
def test_plan_host_spawn_consumes_np_random_like_reference(name):
    """spawn.plan_spawn draws (distance, bearing) per waypoint from the legacy global
    np.random like plan_waypoint_env.py:205-206: seeding it reproduces the golden rows."""
    g = dict(np.load(f"{GOLD}/{name}.npz"))
    np.random.seed(int(g["seed"]))
    for ep in range(len(g["length"])):
        assert np.array_equal(spawn.plan_spawn(), g["spawn"][ep])


def test_host_spawn_with_same_step_is_rejected():
    """SAME_STEP respawns inside the step kernel, before the host knows which envs end, so
    reference-order host spawn rows cannot be supplied: refused up front."""
    from bluesky_gym import _native as nat
    from bluesky_gym.vector import MergeVectorEnv
    with pytest.raises(ValueError, match="NEXT_STEP"):
        MergeVectorEnv(num_envs=4, spawn="host", autoreset=nat.AUTORESET_SAME_STEP)
