"""Extract the reference's saved SAC actors and the tails of its SAC training logs.

Run in the build container only (needs /root/reference):

    python tests/golden/extract_sac_actors.py

Sources (reference-held artefacts, read as data only):
- ``scripts/common/results/models_backup/<Env>/<Env>_SAC/model.zip``: only the member
  ``policy.pth`` is read, with ``torch.load(weights_only=True)`` (no unpickling); the
  ``data`` member is read as JSON text for the observation-space key order and is never
  deserialised further.  The actor is SB3's SAC ``Actor`` (stable-baselines3 2.2.1, the
  version in the archive's ``system_info.txt``): ``latent_pi`` = Linear-ReLU-Linear-ReLU
  (256, 256), ``mu`` and ``log_std`` heads; MultiInputPolicy's CombinedExtractor feeds
  the Dict observation flattened in sorted-key order (the same order as this build's
  ``obs`` rows).
- ``scripts/common/results/logs_backup/<Env>/<Env>_SAC.csv``: the per-episode rows that
  ``scripts/common/logger.py:15-36`` wrote during training (info dict of env 0 at every
  ``done``); the last ``TAIL`` rows are kept, plus the episode length recovered from the
  ``timesteps`` column (one env: consecutive done timesteps differ by the length).

Output: ``tests/golden/sac_actors.npz`` (float32 weights, float64 log columns; numeric
arrays only).
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
ENVS = {"DescentEnv-v0": "descent", "VerticalCREnv-v0": "vertical",
        "HorizontalCREnv-v0": "horizontal", "PlanWaypointEnv-v0": "plan",
        "StaticObstacleEnv-v0": "static", "SectorCREnv-v0": "sector"}
ACTOR_KEYS = ("latent_pi.0.weight", "latent_pi.0.bias", "latent_pi.2.weight",
              "latent_pi.2.bias", "mu.weight", "mu.bias", "log_std.weight", "log_std.bias")


def _obs_keys(data_json: str):
    """Key order of the saved observation space (its repr string in the JSON 'data')."""
    spaces = json.loads(data_json)["observation_space"]["spaces"]
    keys = []
    for part in spaces.split("('")[1:]:
        keys.append(part.split("'", 1)[0])
    return keys


def main():
    import torch
    out = {}
    for env, tag in ENVS.items():
        with zipfile.ZipFile(f"{REF}/models_backup/{env}/{env}_SAC/model.zip") as z:
            sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True,
                            map_location="cpu")
            keys = _obs_keys(z.read("data").decode())
        assert keys == sorted(keys), (env, keys)
        for k in ACTOR_KEYS:
            out[f"{tag}/{k}"] = sd[f"actor.{k}"].float().numpy()
        with open(f"{REF}/logs_backup/{env}/{env}_SAC.csv") as f:
            rows = list(csv.reader(f))
        head, body = rows[0], rows[1:]
        ts = np.array([float(r[0]) for r in body])
        length = np.diff(ts, prepend=0.0)
        for j, name in enumerate(head):
            if name in ("timesteps", "episodes"):
                continue
            col = []
            for r in body[-TAIL:]:
                v = r[j]
                col.append(1.0 if v == "True" else 0.0 if v == "False" else
                           float(v) if v not in ("", "nan") else np.nan)
            out[f"{tag}/log/{name}"] = np.array(col, np.float64)
        out[f"{tag}/log/length"] = length[-TAIL:]
        out[f"{tag}/obs_dim"] = np.array(sd["actor.latent_pi.0.weight"].shape[1])
        print(env, "obs", out[f"{tag}/obs_dim"], "keys", len(keys),
              {k[len(tag) + 5:]: round(float(np.nanmean(v)), 4)
               for k, v in out.items() if k.startswith(f"{tag}/log/")})
    np.savez_compressed(os.path.join(HERE, "sac_actors.npz"), **out)


if __name__ == "__main__":
    main()
