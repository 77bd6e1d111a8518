"""Distributional pin of the device sim layer: the reference's saved SAC actors drive
4,096 device envs each (one episode per env, stochastic actions sampled on the device,
torch fp32 forward on the kernel's own obs rows -- the learner hand-off of SURVEY
§8(f)2) and the episode statistics must match the reference's SAC training logs
(logs_backup/*_SAC.csv, last 1,000 episodes) within sac_policy.BAND standard errors:
episode length, total reward, final altitude (descent_env.py:128-144), intrusions
(vertical_cr_env.py:233-239, horizontal_cr_env.py:260-270), drift, truncation.

These statistics move with the sim-layer decisions of docs/BLUESKY_SUBSET_SPEC.md A.3
(speed envelope: episode length; vertical-speed limit: Descent's final altitude;
phase-GD envelope: Horizontal / PlanWaypoint lengths), which no reference fixture pins
value by value."""
import numpy as np
import pytest
import torch

import sac_policy as sp

pytestmark = pytest.mark.gpu

E = 4096


def _cfg(tag):
    from bluesky_gym import config
    return {"descent": config.descent_config, "vertical": config.vertical_config,
            "horizontal": config.horizontal_config,
            "plan": config.plan_waypoint_config}[tag]()


def rollout_device(tag, W, seed=3):
    from bluesky_gym import core
    b = core.DeviceBatch(_cfg(tag), E, compute_cd=False, seed=seed)
    actor = sp.TorchActor(W, tag, b.device)
    gen = torch.Generator(device=b.device)
    gen.manual_seed(seed)
    obs = b.reset()
    done_once = torch.zeros(E, dtype=torch.bool, device=b.device)
    length = torch.zeros(E, dtype=torch.float64, device=b.device)
    info = torch.zeros((E, 4), dtype=torch.float64, device=b.device)
    trunc_at = torch.zeros(E, dtype=torch.float64, device=b.device)
    for t in range(400):
        with torch.no_grad():
            a = actor(obs, gen)
        obs, _, term, trunc = b.step(a)
        live = ~done_once
        length += live.double()
        d = (term.bool() | trunc.bool()) & live
        info = torch.where(d[:, None], b.ep_info, info)
        trunc_at = torch.where(d, (trunc.bool() & ~term.bool()).double(), trunc_at)
        done_once |= d
        if t % 10 == 9 and bool(done_once.all()):
            break
    assert bool(done_once.all()), f"{tag}: not every env finished an episode"
    info, trunc_at, length = info.cpu().numpy(), trunc_at.cpu().numpy(), length.cpu().numpy()
    rec = {k: np.array([sp.info_row(tag, info[i], trunc_at[i])[k] for i in range(E)])
           for k in sp.LOG_KEYS[tag]}
    rec["length"] = length
    return rec


@pytest.mark.parametrize("tag", ["descent", "vertical", "horizontal", "plan"])
def test_device_reproduces_reference_sac_logs(tag):
    W = sp.load()
    rec = rollout_device(tag, W)
    lines, bad = sp.compare(W, tag, rec)
    print("\n".join(lines))
    assert not bad, f"{tag}: outside {sp.BAND} SE of the reference log: {bad}\n" + "\n".join(lines)
