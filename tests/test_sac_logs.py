"""Distributional pin of the sim layer on the CPU oracle: the reference's saved SAC actors
(scripts/common/results/models_backup/*_SAC/model.zip) rolled out on oracle/ reproduce the
episode statistics their own training logs recorded (logs_backup/*_SAC.csv, last 1,000
episodes) -- episode length, total reward, final altitude / intrusions / drift.  The
envelope constants VMAX_CAS, VSMAX and the phase-GD envelope in oracle/bluesky_subset.py
are fitted to these logs; the device path is checked the same way in
tests/test_gpu_sac_logs.py."""
import numpy as np
import pytest

import sac_policy as sp
from oracle import batched as ob

CASES = {"descent": (lambda E: ob.DescentOracle(E, seed=5), 1500),
         "vertical": (lambda E: ob.VerticalOracle(E, seed=5), 800),
         "horizontal": (lambda E: ob.HorizontalOracle(E, seed=5), 400)}


def rollout_oracle(o, tag, W, E, seed=0):
    """Each env's first episode under the stochastic actor (NEXT_STEP autoreset)."""
    rng = np.random.default_rng(seed)
    obs = o.reset()["obs"]
    done_once = np.zeros(E, bool)
    length = np.zeros(E)
    rec = {}
    for _ in range(400):
        r = o.step(sp.actor_np(W, tag, obs, rng))
        obs = r["obs"]
        live = ~done_once & ~r["was_reset"]
        length[live] += 1
        d = (r["terminated"] | r["truncated"]) & live
        info = o.info()
        info["TimeLimit.truncated"] = r["truncated"] & ~r["terminated"]
        for k in sp.LOG_KEYS[tag]:
            rec.setdefault(k, np.full(E, np.nan))[d] = np.asarray(info[k], np.float64)[d]
        done_once |= d
        if done_once.all():
            break
    assert done_once.all()
    rec["length"] = length
    return rec


@pytest.mark.parametrize("tag", sorted(CASES))
def test_oracle_reproduces_reference_sac_logs(tag):
    W = sp.load()
    make, E = CASES[tag]
    rec = rollout_oracle(make(E), tag, W, E)
    lines, bad = sp.compare(W, tag, rec)
    print("\n".join(lines))
    assert not bad, f"{tag}: outside {sp.BAND} SE of the reference log: {bad}\n" + "\n".join(lines)


def test_fixture_holds_the_logged_tails():
    W = sp.load()
    for tag in sp.LOG_KEYS:
        assert W[f"{tag}/log/length"].shape == (1000,)
        assert W[f"{tag}/latent_pi.0.weight"].shape[1] == int(W[f"{tag}/obs_dim"])
    # Descent: last 1,000 episodes of DescentEnv-v0_SAC.csv (VERDICT r01 figures)
    assert abs(W["descent/log/total_reward"].mean() - (-22.211)) < 1e-3
    assert abs(W["descent/log/length"].mean() - 40.576) < 1e-9
