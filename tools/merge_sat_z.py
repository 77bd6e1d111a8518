"""the z statistics the Merge CAS-100 regression bounds guard
(tests/ref_policy.py MERGE_SAT_Z_BOUNDS), measured on the runs they guard over several
seeds -- the oracle's (tests/test_ref_logs.py: 2,048 envs) here on the CPU and the device's
(tests/test_gpu_ref_logs.py: 4,096 envs) on the GPU box.

    python tools/merge_sat_z.py oracle [seeds...]   > profiles/r06/merge_sat_z_oracle.json
    python tools/merge_sat_z.py device [seeds...]   > profiles/r06/merge_sat_z_device.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "bluesky-gym-hallucination_amd"), os.path.join(REPO, "tests")]
import ref_policy as sp  # noqa: E402


def zs(ours):
    """z of each statistic against each log, as merge_sat_compare computes it."""
    L = sp.merge_logs()
    out = {}
    for alg in ("ddpg", "td3"):
        for k in sp.MERGE_SAT_KEYS:
            x, y = np.asarray(ours[k], np.float64), L[f"{alg}/{k}"]
            se = np.hypot(x.std() / np.sqrt(len(x)), sp.bootstrap_se(y))
            out[f"{alg}/{k}"] = float((x.mean() - y.mean()) / se)
    return out


def oracle_run(seed, ac_spd=100, E=2048):
    from oracle import batched as ob
    o = ob.MergeOracle(E, num_ac=20, seed=seed, compute_cd=False, ac_spd=ac_spd)
    o.reset()
    act = np.tile([1.0, 1.0], (E, 1))
    for _ in range(50):
        r = o.step(act)
    assert r["truncated"].all()
    info = o.info()
    return {k: info[k] for k in sp.MERGE_SAT_KEYS}


def device_run(seed, ac_spd=100, E=4096):
    import torch
    from bluesky_gym import config, core
    b = core.DeviceBatch(config.merge_config(num_ac=20, ac_spd=ac_spd), E, seed=seed)
    b.reset()
    act = torch.ones((E, 2), dtype=torch.float64, device=b.device)
    for _ in range(50):
        b.step(act)
    assert bool(b.truncated.bool().all())
    info = b.ep_info.cpu().numpy()
    return {"total_reward": info[:, 0], "total_intrusions": info[:, 1], "average_drift": info[:, 3]}


def main():
    mode = sys.argv[1]
    seeds = [int(s) for s in sys.argv[2:]] or ([11, 12, 13, 14, 15, 16] if mode == "oracle"
                                               else [7, 8, 9, 10, 11, 12, 13, 14])
    run = oracle_run if mode == "oracle" else device_run
    rows = {}
    for s in seeds:
        rows[s] = zs(run(s))
        print(f"seed {s}: " + "  ".join(f"{k} {v:+.2f}" for k, v in rows[s].items()),
              file=sys.stderr, flush=True)
    keys = list(next(iter(rows.values())))
    summ = {k: [min(r[k] for r in rows.values()), max(r[k] for r in rows.values())] for k in keys}
    print(json.dumps({"mode": mode, "ac_spd": 100, "envs": 2048 if mode == "oracle" else 4096,
                      "seeds": rows, "range": summ}, indent=1))


if __name__ == "__main__":
    main()
