"""Distributional pin of the sim layer on the CPU oracle: the reference's saved actors
(scripts/common/results/models_backup/*/model.zip) rolled out on oracle/ reproduce the
episode statistics their own training logs recorded (logs_backup/*.csv, last 1,000
episodes) -- episode length, total reward, final altitude / intrusions / drift / crashes.

Two groups (tests/ref_policy.py):
- the SAC actors of Descent / Vertical / Horizontal: the envelope constants VMAX_CAS,
  VSMAX and the phase-GD envelope in oracle/bluesky_subset.py were fitted to some of these
  statistics (ref_policy.FITTED, bar BAND_FIT); the rest are held out;
- HELD-OUT actors never used for any fit, with the constants frozen: the DDPG (Descent,
  PlanWaypoint) and PPO (Vertical, Horizontal, StaticObstacle, SectorCR) actors, and the
  StaticObstacle / SectorCR SAC actors; bar BAND_HELDOUT.  Statistics outside it are
  listed in ref_policy.KNOWN_RED with the decision that moves them; any other red
  statistic fails.  (The PlanWaypoint / StaticObstacle SAC rollouts run on the device
  only, tests/test_gpu_ref_logs.py: 240-step episodes / the oracle's per-env polygon
  loop are slow here.)

The device path is checked the same way, with 4,096 envs per case, in
tests/test_gpu_ref_logs.py."""
import numpy as np
import pytest

import ref_policy as sp
from oracle import batched as ob
from oracle import batched_areas as oba

MAKERS = {"descent": lambda E: ob.DescentOracle(E, seed=5),
          "vertical": lambda E: ob.VerticalOracle(E, seed=5),
          "horizontal": lambda E: ob.HorizontalOracle(E, seed=5),
          "plan": lambda E: ob.PlanWaypointOracle(E, seed=5),
          "static": lambda E: oba.StaticOracle(E, seed=5),
          "sector": lambda E: oba.SectorOracle(E, seed=5, compute_cd=False)}
# PlanWaypoint keeps a truncated episode's aircraft (plan_waypoint_env.py:156-171), and
# its logs are a long run of consecutive episodes: compare each env's second episode,
# which starts from the first one's end state when that one was truncated.
EPISODE = {"plan": 1}
# tag -> envs in the CPU rollout
CASES = {"descent": 1500, "vertical": 800, "horizontal": 400,
         "descent_ddpg": 1500, "vertical_ppo": 800, "horizontal_ppo": 400,
         "sector": 200, "sector_ppo": 200, "plan_ddpg": 300, "static": 60, "static_ppo": 60}


def rollout_oracle(o, tag, W, E, seed=0, horizon=None):
    """Each env's first episode (EPISODE[env]-th, counting from 0) under the actor as its
    training run drew actions (SAC / PPO sampled, DDPG deterministic), NEXT_STEP
    autoreset."""
    env = sp.env_of(tag)
    want = EPISODE.get(env, 0)
    horizon = horizon or 400 * (want + 1)
    rng = None if sp.alg_of(W, tag) == "ddpg" else np.random.default_rng(seed)
    obs = o.reset()["obs"]
    ndone = np.zeros(E, np.int64)
    length = np.zeros(E)
    rec = {}
    for _ in range(horizon):
        r = o.step(sp.actor_np(W, tag, obs, rng))
        obs = r["obs"]
        live = (ndone == want) & ~r["was_reset"]
        length[live] += 1
        d = (r["terminated"] | r["truncated"]) & ~r["was_reset"]
        info = o.info()
        info["TimeLimit.truncated"] = r["truncated"] & ~r["terminated"]
        for k in sp.LOG_KEYS[env]:
            rec.setdefault(k, np.full(E, np.nan))[d & live] = np.asarray(info[k], np.float64)[d & live]
        ndone += d
        if (ndone > want).all():
            break
    assert (ndone > want).all()
    rec["length"] = length
    return rec


@pytest.mark.parametrize("tag", sorted(CASES))
def test_oracle_reproduces_reference_logs(tag):
    W = sp.load()
    E = CASES[tag]
    rec = rollout_oracle(MAKERS[sp.env_of(tag)](E), tag, W, E)
    lines, bad, rows = sp.compare(W, tag, rec)
    print("\n".join(sp.annotate(lines, rows)))
    unexpected = [k for k in bad if (tag, k) not in sp.KNOWN_RED]
    assert not unexpected, (f"{tag}: outside its band of the reference log: {unexpected}\n"
                            + "\n".join(lines))


def test_fixture_holds_the_logged_tails():
    W = sp.load()
    for tag in sp.SAC_TAGS + sp.HELDOUT_TAGS:
        assert W[f"{tag}/log/length"].shape == (1000,)
        if sp.alg_of(W, tag) == "sac":
            assert W[f"{tag}/latent_pi.0.weight"].shape[1] == int(W[f"{tag}/obs_dim"])
    # Descent: last 1,000 episodes of DescentEnv-v0_SAC.csv (VERDICT r01 figures)
    assert abs(W["descent/log/total_reward"].mean() - (-22.211)) < 1e-3
    assert abs(W["descent/log/length"].mean() - 40.576) < 1e-9
    # held-out logs (extract_ref_actors.py)
    assert abs(W["descent_ddpg/log/length"].mean() - 40.564) < 1e-9
    assert abs(W["static_ppo/log/crashed"].mean() - 0.421) < 1e-9
    # the StaticObstacle logs carry no drift term (integer rewards, NaN average_drift)
    for tag in ("static", "static_ppo"):
        r = W[f"{tag}/log/total_reward"]
        assert np.array_equal(r, np.round(r)) and np.isnan(W[f"{tag}/log/average_drift"]).all()


def test_actor_forms():
    """DDPG is deterministic and squashed; PPO samples around its mean and clips."""
    W = sp.load()
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64, int(W["descent_ddpg/obs_dim"])))
    a = sp.actor_np(W, "descent_ddpg", x)
    assert np.all(np.abs(a) <= 1) and np.array_equal(a, sp.actor_np(W, "descent_ddpg", x, rng))
    x = rng.standard_normal((4096, int(W["static_ppo/obs_dim"])))
    m = sp.actor_np(W, "static_ppo", x)
    s = sp.actor_np(W, "static_ppo", x, np.random.default_rng(2))
    assert s.shape == (4096, 2) and s.min() == -1.0 and s.max() == 1.0   # std ~1.8: clipped
    assert np.abs(m).max() <= 1.0


@pytest.mark.parametrize("ac_spd", [100, 150])
def test_merge_saturated_policy(ac_spd):
    """MergeEnv-v0's own DDPG / TD3 logs: from episode 3 on a constant
    (+-1, +1) action flew them -- HDG +-15 deg and SPD +20 m/s every RL step
    (merge_env.py:286-293), a circling ownship, every episode truncated at 50 steps.  The
    statistics pin the sim layer under the headline env: the intruders' spawn and LNAV
    stream (merge_env.py:148-158, FIX then RWY), the ownship's speed envelope at 10,000 m
    and the intrusion count (:275-284).  num_ac = 20, the env's default.  Compared with both
    logs' last 1,000 episodes: drift mean / spread, intrusions, reward and the intrusion
    histogram; the known reds (ref_policy.KNOWN_RED) carry the decision that moves them."""
    E = 2048
    o = ob.MergeOracle(E, num_ac=20, seed=11, compute_cd=False, ac_spd=ac_spd)
    o.reset()
    act = np.tile([1.0, 1.0], (E, 1))
    for _ in range(50):
        r = o.step(act)
    assert r["truncated"].all()
    info = o.info()
    tag = f"merge_sat_{ac_spd}"
    lines, bad = sp.merge_sat_compare(tag, {k: info[k] for k in sp.MERGE_SAT_KEYS})
    print("\n".join(lines))
    unexpected = [k for k in bad if (tag, k) not in sp.KNOWN_RED]
    assert not unexpected, f"{tag}: outside its band of the reference logs: {unexpected}\n" + "\n".join(lines)
