"""Extract the observations the reference's saved models hold as text (the sim-layer pins of
DESIGN.md §5: the Merge cruise-speed cap, and the one-step transitions of the off-policy
models).

Run in the build container only (reads /root/reference):

    python tests/golden/extract_last_obs.py

Each ``scripts/common/results/models_backup/<Env>/<Env>_<ALG>/model.zip`` carries a ``data``
member that is plain JSON (stable-baselines3's ``save``).  Its ``_last_obs`` -- and for the
off-policy algorithms ``_last_original_obs`` -- are dicts whose per-key values are the
``str()`` of a NumPy array (8 decimals, NumPy's default print precision), next to a
``:serialized:`` pickle of the same object.  Only ``zipfile`` + ``json`` + ``float()`` touch
the file; the pickles are never read.

Without a VecNormalize wrapper (none of the reference scripts uses one,
``scripts/*_sac.py``, ``main.py``) SB3's off-policy ``_store_transition`` sets
``_last_original_obs = _last_obs`` and then ``_last_obs = new_obs``: so for SAC / DDPG /
TD3 the pair (``_last_original_obs``, ``_last_obs``) is one env step of the reference's
simulator -- the observation before and after the last training step (or a reset, when that
step ended the episode).

Output: tests/golden/last_obs.npz with keys ``<Env>/<ALG>/<which>/<obs key>`` (float64
arrays of the printed values), ``<Env>/<ALG>/num_timesteps`` and ``<Env>/<ALG>/n_envs``.
"""
from __future__ import annotations

import glob
import json
import os
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MODELS = "/root/reference/scripts/common/results/models_backup"


def parse_printed(text: str) -> np.ndarray:
    """'[[0.1 -0.2\\n  0.3]]' -> array([0.1, -0.2, 0.3]) (float() of each printed token)."""
    toks = text.replace("[", " ").replace("]", " ").split()
    return np.array([float(t) for t in toks], np.float64)


def main():
    out = {}
    for path in sorted(glob.glob(os.path.join(MODELS, "*", "*", "model.zip"))):
        env, run = path.split(os.sep)[-3:-1]
        alg = run.split("_")[-1]
        with zipfile.ZipFile(path) as z:
            data = json.loads(z.read("data"))
        tag = f"{env}/{alg}"
        out[f"{tag}/num_timesteps"] = np.array(int(data["num_timesteps"]))
        out[f"{tag}/n_envs"] = np.array(int(data["n_envs"]))
        for which in ("_last_obs", "_last_original_obs"):
            d = data.get(which)
            if not isinstance(d, dict):
                continue
            for k, v in d.items():
                if k.startswith(":"):
                    continue                      # ':type:' text, ':serialized:' pickle
                out[f"{tag}/{which.strip('_')}/{k}"] = parse_printed(v)
    np.savez_compressed(os.path.join(HERE, "last_obs.npz"), **out)
    for k, v in out.items():
        print(k, np.array2string(np.atleast_1d(v), precision=8, max_line_width=200))


if __name__ == "__main__":
    main()
