"""GPU checks of the drop-in API: gym.make single envs reproduce the reference's golden
episodes when Python random / np.random are seeded as the reference consumes them;
gym.make_vec vector envs; the SB3 VecEnv adapter; shard equivalence for multi-GPU."""
import os
import random

import numpy as np
import pytest
import torch

import bluesky_gym
from bluesky_gym import _gym
from bluesky_gym import _native as nat
from bluesky_gym.obs_layout import ObsLayout
import oracle_replay as rp

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def flat(obs, keys):
    return np.concatenate([np.asarray(obs[k], np.float64).ravel() for k in keys])


def close(a, b):
    return np.all(np.abs(np.asarray(a) - np.asarray(b)) <= 1e-5 + 1e-5 * np.abs(np.asarray(b)))


def test_gym_make_merge_reproduces_reference_episode():
    import bluesky_gym.envs.merge_env as me
    bluesky_gym.register_envs()
    g = dict(np.load(f"{GOLD}/merge_N8.npz"))
    me.NUM_AC = 8                       # the reference is patched the same way (make_golden.py)
    try:
        random.seed(0)
        env = _gym.make("MergeEnv-v0")
        keys = ObsLayout(nat.ENV_MERGE, 8, 5).keys
        for ep in range(len(g["length"])):
            obs, info = env.reset()
            assert close(flat(obs, keys), g["obs0"][ep])
            assert np.isnan(info["average_drift"])
            for t in range(g["length"][ep]):
                obs, rew, term, trunc, info = env.step(g["actions"][ep, t])
                assert close(flat(obs, keys), g["obs"][ep, t]), (ep, t)
                assert abs(rew - g["reward"][ep, t]) <= 1e-5 + 1e-5 * abs(g["reward"][ep, t])
                assert term == g["terminated"][ep, t] and trunc == bool(g["truncated"][ep, t])
                assert isinstance(term, int)
            assert abs(info["total_reward"] - g["info"][ep, t, 0]) < 1e-9
            assert info["total_intrusions"] == g["info"][ep, t, 3]
        env.close()
    finally:
        me.NUM_AC = 20


def test_gym_make_vertical_and_descent_reproduce_reference():
    bluesky_gym.register_envs()
    for name, eid, seed, kw in (("vertical_N6", "VerticalCREnv-v0", 4, {}),
                                ("descent", "DescentEnv-v0", 6, {}),
                                ("horizontal_N6", "HorizontalCREnv-v0", 7, {})):
        g = dict(np.load(f"{GOLD}/{name}.npz"))
        np.random.seed(seed)
        env = _gym.make(eid, **kw)
        keys = sorted(env.observation_space.spaces)
        for ep in range(len(g["length"])):
            obs, _ = env.reset()
            assert close(flat(obs, keys), g["obs0"][ep])
            for t in range(g["length"][ep]):
                obs, rew, term, trunc, info = env.step(g["actions"][ep, t])
                assert close(flat(obs, keys), g["obs"][ep, t]), (name, ep, t)
                assert term == g["terminated"][ep, t]
        env.close()


def test_make_vec_merge_batch_and_autoreset():
    bluesky_gym.register_envs()
    E = 512
    venv = _gym.make_vec("MergeEnv-v0", num_envs=E, vectorization_mode="vector_entry_point",
                         num_ac=32, seed=3)
    obs, info = venv.reset()
    assert obs["x_r"].shape == (E, 5) and obs["airspeed"].shape == (E, 1)
    rng = np.random.default_rng(0)
    seen_done = np.zeros(E, bool)
    for t in range(55):
        obs, rew, term, trunc, info = venv.step(rng.uniform(-1, 1, (E, 2)))
        assert rew.shape == (E,) and term.dtype == bool
        if t == 49:
            assert (term | trunc).all() or trunc.sum() > 0
        if t == 50:
            # NEXT_STEP: the step after done resets with reward 0 and no termination
            assert np.all(rew[seen_done] == 0.0)
        seen_done = term | trunc
    venv.close()


def test_sb3_vecenv_terminal_observation_and_infos():
    from bluesky_gym.sb3 import SB3VecEnv
    E = 256
    env = SB3VecEnv("MergeEnv-v0", E, num_ac=32, seed=9)
    obs = env.reset()
    assert set(obs) == set(env.observation_space.spaces)
    rng = np.random.default_rng(1)
    got_terminal = False
    for t in range(52):
        obs, rew, dones, infos = env.step(rng.uniform(-1, 1, (E, 2)))
        assert len(infos) == E and set(("total_reward", "faf_reach", "average_drift",
                                        "total_intrusions")) <= set(infos[0])
        for i in np.nonzero(dones)[0]:
            to = infos[i]["terminal_observation"]
            assert set(to) == set(obs) and "TimeLimit.truncated" in infos[i]
            got_terminal = True
    assert got_terminal
    env.close()


@pytest.mark.parametrize("env_id,kw,A", [("MergeEnv-v0", dict(num_ac=32, max_episode_steps=12), 2),
                                         ("DescentEnv-v0", dict(max_episode_steps=15), 1),
                                         ("PlanWaypointEnv-v0", dict(max_episode_steps=15), 1)])
def test_rllib_vector_env_matches_sb3_adapter(env_id, kw, A):
    """RLlib's legacy VectorEnv contract on the device batch: vector_step reports a finished
    env's terminal observation and reset_at(i) its next episode's first observation -- the
    same values SB3's adapter reports as infos["terminal_observation"] and obs on the same
    seed (both run SAME_STEP autoreset on one kernel); episode infos agree."""
    from bluesky_gym.rllib import RLlibVectorEnv
    from bluesky_gym.sb3 import SB3VecEnv
    E = 128
    rl = RLlibVectorEnv(env_id, E, seed=4, **kw)
    sb = SB3VecEnv(env_id, E, seed=4, **kw)
    obs_rl, infos = rl.vector_reset()
    obs_sb = sb.reset()
    keys = sorted(obs_sb)
    assert len(obs_rl) == E and len(infos) == E
    for i in (0, E - 1):
        assert np.array_equal(flat(obs_rl[i], keys), flat({k: v[i] for k, v in obs_sb.items()}, keys))
    rng = np.random.default_rng(6)
    n_done = 0
    for t in range(40):
        a = rng.uniform(-1, 1, (E, A))
        o_rl, r_rl, te, tr, inf_rl = rl.vector_step(a)
        o_sb, r_sb, d_sb, inf_sb = sb.step(a)
        assert np.array_equal(np.asarray(r_rl, np.float32), r_sb)
        assert np.array_equal(np.asarray(te) | np.asarray(tr), d_sb)
        for i in range(E):
            if d_sb[i]:
                n_done += 1
                assert np.array_equal(flat(o_rl[i], keys), flat(inf_sb[i]["terminal_observation"], keys))
                assert inf_rl[i]["total_reward"] == inf_sb[i]["total_reward"]
                o_new, _ = rl.reset_at(i)
                assert np.array_equal(flat(o_new, keys), flat({k: v[i] for k, v in o_sb.items()}, keys))
            elif i % 17 == 0:
                assert np.array_equal(flat(o_rl[i], keys), flat({k: v[i] for k, v in o_sb.items()}, keys))
    assert n_done > 0
    # an env that did not finish is reset by a masked reset launch
    o5, _ = rl.reset_at(5)
    assert all(np.all(np.isfinite(v)) for v in o5.values())
    assert int(rl.venv.batch.envs["step_count"][5]) == 0
    rl.close()
    sb.close()


def test_shards_equal_one_big_batch():
    """Global env ids (env_offset) make two 128-env shards identical to one 256 batch."""
    from bluesky_gym import config, core
    cfg = config.merge_config(num_ac=32)
    big = core.DeviceBatch(cfg, 256, seed=21)
    s0 = core.DeviceBatch(cfg, 128, seed=21, env_offset=0)
    s1 = core.DeviceBatch(cfg, 128, seed=21, env_offset=128)
    big.reset(); s0.reset(); s1.reset()
    rng = np.random.default_rng(2)
    for t in range(60):
        a = torch.from_numpy(rng.uniform(-1, 1, (256, 2)))
        big.step(a); s0.step(a[:128]); s1.step(a[128:])
        cat = torch.cat([s0.obs, s1.obs]).cpu()
        assert torch.equal(big.obs.cpu(), cat)
        assert torch.equal(big.conf_mask.cpu(), torch.cat([s0.conf_mask, s1.conf_mask]).cpu())
