"""Extract the reference's saved DDPG and PPO actors with the tails of their own training
logs: the held-out check of the fitted sim-layer envelope.  The SAC actors,
to which VMAX_CAS / VSMAX / the phase-GD envelope were fitted, are in sac_actors.npz
(extract_sac_actors.py); nothing here was used for that fit.

Run in the build container only (needs /root/reference):

    python tests/golden/extract_ref_actors.py

Sources (reference-held artefacts, read as data only):
- ``scripts/common/results/models_backup/<Env>/<Env>_<ALG>/model.zip``: only the member
  ``policy.pth`` is read, with ``torch.load(weights_only=True)`` (no unpickling); the
  ``data`` member is read as JSON text for the observation-space key order and the
  hyper-parameters that decide how the training run drew its actions (``action_noise``,
  ``use_sde``), and is never deserialised further.  stable-baselines3 2.2.1 (the
  archives' ``system_info.txt``):
  * DDPG ``Actor``: ``mu`` = Linear-ReLU-Linear-ReLU-Linear-Tanh (400, 300); trained with
    ``action_noise=None``, so the logged episodes were flown by the deterministic
    ``tanh(mu(obs))`` of the actor of the moment;
  * PPO ``ActorCriticPolicy``: ``mlp_extractor.policy_net`` = Linear-Tanh-Linear-Tanh (64,
    64), ``action_net``, state-independent ``log_std``; training samples
    ``N(mean, exp(log_std))`` and clips the sample to the Box before ``env.step``
    (``OnPolicyAlgorithm.collect_rollouts``).
- ``scripts/common/results/logs_backup/<Env>/<Env>_<ALG>.csv``: the per-episode rows
  ``scripts/common/logger.py:15-36`` wrote during training; the last ``TAIL`` rows, plus
  the episode length from the ``timesteps`` column.

Pairs with no actor or no log in the reference are not extractable: MergeEnv-v0 holds
PPO/SAC actors whose logs are listed in ``.MISSING_LARGE_BLOBS`` and DDPG/TD3 logs whose
actors are missing, so Merge's sim layer stays unpinned by this route.

Output: ``tests/golden/ref_actors.npz`` (float32 weights, float64 log columns, a
``<tag>/alg`` string; numeric/unicode arrays only, loads with allow_pickle=False).
"""
from __future__ import annotations

import csv
import io
import json
import os
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/scripts/common/results"
TAIL = 1000
# tag -> (env id, algorithm)
PAIRS = {"descent_ddpg": ("DescentEnv-v0", "DDPG"),
         "plan_ddpg": ("PlanWaypointEnv-v0", "DDPG"),
         "vertical_ppo": ("VerticalCREnv-v0", "PPO"),
         "horizontal_ppo": ("HorizontalCREnv-v0", "PPO"),
         "static_ppo": ("StaticObstacleEnv-v0", "PPO"),
         "sector_ppo": ("SectorCREnv-v0", "PPO")}
KEYS = {"DDPG": ("actor.mu.0.weight", "actor.mu.0.bias", "actor.mu.2.weight",
                 "actor.mu.2.bias", "actor.mu.4.weight", "actor.mu.4.bias"),
        "PPO": ("mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
                "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
                "action_net.weight", "action_net.bias", "log_std")}


def _obs_keys(data_json: dict):
    spaces = data_json["observation_space"]["spaces"]
    return [part.split("'", 1)[0] for part in spaces.split("('")[1:]]


def _log_tail(path):
    with open(path) as f:
        rows = list(csv.reader(f))
    head, body = rows[0], rows[1:]
    ts = np.array([float(r[0]) for r in body])
    length = np.diff(ts, prepend=0.0)
    out = {}
    for j, name in enumerate(head):
        if name in ("timesteps", "episodes"):
            continue
        col = []
        for r in body[-TAIL:]:
            v = r[j]
            col.append(1.0 if v == "True" else 0.0 if v == "False" else
                       float(v) if v not in ("", "nan") else np.nan)
        out[name] = np.array(col, np.float64)
    out["length"] = length[-TAIL:]
    return out


def main():
    import torch
    out = {}
    for tag, (env, alg) in PAIRS.items():
        with zipfile.ZipFile(f"{REF}/models_backup/{env}/{env}_{alg}/model.zip") as z:
            sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True,
                            map_location="cpu")
            data = json.loads(z.read("data").decode())
        keys = _obs_keys(data)
        assert keys == sorted(keys), (env, keys)
        assert data["action_noise"] is None and not data["use_sde"], (env, alg)
        for k in KEYS[alg]:
            out[f"{tag}/{k}"] = sd[k].float().numpy()
        out[f"{tag}/alg"] = np.array(alg.lower())
        first = KEYS[alg][0]
        out[f"{tag}/obs_dim"] = np.array(sd[first].shape[1])
        for name, col in _log_tail(f"{REF}/logs_backup/{env}/{env}_{alg}.csv").items():
            out[f"{tag}/log/{name}"] = col
        print(env, alg, "obs", int(out[f"{tag}/obs_dim"]),
              {k[len(tag) + 5:]: round(float(np.nanmean(v)), 4)
               for k, v in out.items() if k.startswith(f"{tag}/log/")})
    np.savez_compressed(os.path.join(HERE, "ref_actors.npz"), **out)


if __name__ == "__main__":
    main()
