"""The reference's saved actors and the tails of their own training logs, as a
distributional pin of the BlueSky sim layer (parity of the simulator arithmetic is
otherwise unpinned: bluesky-simulator is not vendored).

Fixtures (numeric arrays; tests/golden/extract_*.py, container-only):
- tests/golden/sac_actors.npz: the SAC actors of all six single-agent-policy envs
  (stable-baselines3 2.2.1 ``Actor``: Linear-ReLU-Linear-ReLU 256/256, ``mu``, ``log_std``
  clamped to [-20, 2], action = tanh(mu + std * eps) while training).  The envelope
  constant VMAX_CAS of oracle/bluesky_subset.py was FITTED to the episode lengths of two
  of these logs (FITTED below): those statistics are in-sample.  (The phase-GD cap, fitted
  to the Horizontal / PlanWaypoint lengths until round 4, is now pinned value by value by
  the saved Horizontal observations, tests/test_last_obs.py; those lengths are held out.)  (The round-2 VSMAX fit to Descent's final altitude was withdrawn in round 4:
  the held-out actors rejected it; that statistic is held out again.)
- tests/golden/ref_actors.npz: the DDPG and PPO actors with their logs
  (extract_ref_actors.py), never used for any fit: HELD-OUT.
  * DDPG ``Actor``: Linear-ReLU 400, Linear-ReLU 300, Linear-Tanh; trained without
    action noise, so the logged episodes were flown by tanh(mu(obs)).
  * PPO: ``policy_net`` Linear-Tanh 64, Linear-Tanh 64, ``action_net``, state-independent
    ``log_std``; the training run sampled N(mean, exp(log_std)) and clipped it to [-1, 1].

The logged episodes were produced by the policy while it was still being trained; the
saved actor is the final one, so the comparison is statistical: each compared mean is
reported as z = (ours - log) / SE (bootstrap SE of the log, normal SE of the rollout, in
quadrature).  Bars: BAND_FIT on the fitted statistics, BAND_HELDOUT on everything else.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BAND_FIT = 4.0
BAND_HELDOUT = 3.0
BAND = BAND_FIT

# The statistics the fit of docs/BLUESKY_SUBSET_SPEC.md A.3 uses (VMAX_CAS: the Descent /
# Vertical lengths).  Every other (tag, statistic) is held out.
FITTED = {("descent", "length"), ("vertical", "length")}

# info keys compared per env (plus the episode length).  StaticObstacleEnv's logs were
# written by an env revision without the drift term (every logged total_reward is an
# integer, average_drift is NaN in all rows: _check_drift, static_obstacle_env.py:323-327,
# did not run); its reward is then a function of the reach / crash outcome, so the
# outcome flags are compared instead of the reward.
LOG_KEYS = {
    "descent": ("total_reward", "final_altitude"),
    "vertical": ("total_reward", "total_intrusions", "final_altitude"),
    "horizontal": ("total_reward", "total_intrusions", "average_drift"),
    "plan": ("total_reward", "TimeLimit.truncated"),
    "static": ("waypoint_reached", "crashed", "TimeLimit.truncated"),
    "sector": ("total_reward", "total_intrusions", "average_drift"),
}

# Held-out statistics outside BAND_HELDOUT with the envelope frozen, each with what moves
# it (tools/envelope_sensitivity.py sweeps).  They are reported, not hidden:
# a test fails on any red statistic NOT listed here.
_DESCENT_SAC_ALT = ("the one statistic the withdrawn VSMAX fit matched: a vsmax cap of ~12.1 m/s "
                    "on the terminal dive brings it in, and puts Descent DDPG's final altitude at "
                    "z = +15 (held-out evidence against the cap); no single vsmax serves both "
                    "actors' dives.  The saved Descent / Vertical SAC transitions reproduce the "
                    "slew, the integration and CAS->TAS exactly at 860-3,270 m "
                    "(tests/test_last_obs.py), so what is left is the regime below 1,000 ft "
                    "that no saved state reaches (the DDPG's last saved state dives at -12.5 "
                    "m/s at 394 m) (DESIGN.md §5)")
_STATIC = ("logs written by an older StaticObstacleEnv revision (no drift term); not moved by "
           "the A.3 speed envelope")
_SECTOR = ("the logged runs did not fly this Sector state: the saved SAC transition "
           "(tests/test_last_obs.py) has all four intruders at 89.000 m/s, the ground-phase "
           "cap, where sector_cr_env.py:217's CAS 150 at 350 m is 152.4 m/s here, and an ownship "
           "deceleration no axmax-0.5 step gives (DESIGN.md §5); not moved by A.3 vmin / vmax / "
           "bank / vsmax")
_PLAN_DDPG = "not moved by the A.3 phase-GD envelope; the DDPG log tail drifts (last quarter)"
KNOWN_RED = {
    ("descent", "final_altitude"): _DESCENT_SAC_ALT,
    **{(t, k): _STATIC for t in ("static", "static_ppo")
       for k in ("waypoint_reached", "crashed", "TimeLimit.truncated", "length")},
    **{(t, k): _SECTOR for t in ("sector", "sector_ppo")
       for k in ("total_reward", "total_intrusions", "average_drift", "length")},
    **{("plan_ddpg", k): _PLAN_DDPG for k in ("total_reward", "TimeLimit.truncated", "length")},
}

SAC_TAGS = ("descent", "vertical", "horizontal", "plan", "static", "sector")
HELDOUT_TAGS = ("static", "sector", "descent_ddpg", "plan_ddpg", "vertical_ppo",
                "horizontal_ppo", "static_ppo", "sector_ppo")


def load():
    W = dict(np.load(os.path.join(HERE, "golden", "sac_actors.npz")))
    W.update(np.load(os.path.join(HERE, "golden", "ref_actors.npz")))
    return W


def env_of(tag):
    return tag.split("_")[0]


def alg_of(W, tag):
    k = f"{tag}/alg"
    return str(W[k]) if k in W else "sac"


def heldout(tag, stat):
    """True unless (tag, stat) is one of the SAC statistics the envelope was fitted to."""
    return "_" in tag or (env_of(tag), stat) not in FITTED


def actor_np(W, tag, obs, rng=None):
    """The saved actor on float32 observations (SB3 feeds the policy float32); float64
    math.  rng None = the deterministic action (SAC tanh(mu), PPO the mean clipped)."""
    g = lambda k: W[f"{tag}/{k}"].astype(np.float64)  # noqa: E731
    x = np.asarray(obs, np.float32).astype(np.float64)
    alg = alg_of(W, tag)
    if alg == "ddpg":
        h = np.maximum(x @ g("actor.mu.0.weight").T + g("actor.mu.0.bias"), 0.0)
        h = np.maximum(h @ g("actor.mu.2.weight").T + g("actor.mu.2.bias"), 0.0)
        return np.tanh(h @ g("actor.mu.4.weight").T + g("actor.mu.4.bias"))
    if alg == "ppo":
        p = "mlp_extractor.policy_net"
        h = np.tanh(x @ g(f"{p}.0.weight").T + g(f"{p}.0.bias"))
        h = np.tanh(h @ g(f"{p}.2.weight").T + g(f"{p}.2.bias"))
        mean = h @ g("action_net.weight").T + g("action_net.bias")
        if rng is not None:
            mean = mean + np.exp(g("log_std")) * rng.standard_normal(mean.shape)
        return np.clip(mean, -1.0, 1.0)
    h = np.maximum(x @ g("latent_pi.0.weight").T + g("latent_pi.0.bias"), 0.0)
    h = np.maximum(h @ g("latent_pi.2.weight").T + g("latent_pi.2.bias"), 0.0)
    mu = h @ g("mu.weight").T + g("mu.bias")
    if rng is None:
        return np.tanh(mu)
    ls = np.clip(h @ g("log_std.weight").T + g("log_std.bias"), -20.0, 2.0)
    return np.tanh(mu + np.exp(ls) * rng.standard_normal(mu.shape))


class TorchActor:
    """The same actors as torch fp32 modules on a device (the learner-side forward)."""

    def __init__(self, W, tag, device):
        import torch
        self.torch = torch
        self.alg = alg_of(W, tag)
        names = {"sac": ("latent_pi.0.weight", "latent_pi.0.bias", "latent_pi.2.weight",
                         "latent_pi.2.bias", "mu.weight", "mu.bias", "log_std.weight",
                         "log_std.bias"),
                 "ddpg": ("actor.mu.0.weight", "actor.mu.0.bias", "actor.mu.2.weight",
                          "actor.mu.2.bias", "actor.mu.4.weight", "actor.mu.4.bias"),
                 "ppo": ("mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
                         "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
                         "action_net.weight", "action_net.bias", "log_std")}[self.alg]
        self.w = [torch.as_tensor(W[f"{tag}/{k}"], device=device) for k in names]

    def __call__(self, obs, gen=None):
        torch = self.torch
        F = torch.nn.functional
        if self.alg == "ddpg":
            w0, b0, w2, b2, w4, b4 = self.w
            h = F.relu(F.linear(obs, w0, b0))
            h = F.relu(F.linear(h, w2, b2))
            return torch.tanh(F.linear(h, w4, b4))
        if self.alg == "ppo":
            w0, b0, w2, b2, wa, ba, ls = self.w
            h = torch.tanh(F.linear(obs, w0, b0))
            h = torch.tanh(F.linear(h, w2, b2))
            mean = F.linear(h, wa, ba)
            if gen is not None:
                eps = torch.randn(mean.shape, device=mean.device, generator=gen)
                mean = mean + torch.exp(ls) * eps
            return torch.clamp(mean, -1.0, 1.0)
        w0, b0, w2, b2, wm, bm, ws, bs = self.w
        h = F.relu(F.linear(obs, w0, b0))
        h = F.relu(F.linear(h, w2, b2))
        mu = F.linear(h, wm, bm)
        if gen is None:
            return torch.tanh(mu)
        ls = torch.clamp(F.linear(h, ws, bs), -20.0, 2.0)
        eps = torch.randn(mu.shape, device=mu.device, generator=gen)
        return torch.tanh(mu + torch.exp(ls) * eps)


def log_stats(W, tag):
    env = env_of(tag)
    return {k: W[f"{tag}/log/{k}"] for k in LOG_KEYS[env] + ("length",)}


def bootstrap_se(x, reps=2000, seed=0):
    x = np.asarray(x, np.float64)
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, len(x), (reps, len(x)))
    return float(x[idx].mean(axis=1).std())


def compare(W, tag, ours: dict, band_fit=BAND_FIT, band_heldout=BAND_HELDOUT):
    """Per statistic: ours mean, log mean, z, and whether it is a fitted or a held-out
    statistic.  Returns (report lines, statistics outside their band, rows) where a row
    is (tag, stat, kind, ours, log, z)."""
    log = log_stats(W, tag)
    lines, bad, rows = [], [], []
    for k, lv in log.items():
        ov = np.asarray(ours[k], np.float64)
        se = np.hypot(bootstrap_se(lv), ov.std() / np.sqrt(len(ov)))
        z = (ov.mean() - lv.mean()) / max(se, 1e-12)
        kind = "held-out" if heldout(tag, k) else "fitted"
        band = band_heldout if kind == "held-out" else band_fit
        lines.append(f"{tag:15s} {k:20s} {kind:8s} ours {ov.mean():10.4f} (n={len(ov)})  "
                     f"log {lv.mean():10.4f}  z {z:+.2f}")
        rows.append((tag, k, kind, float(ov.mean()), float(lv.mean()), float(z)))
        if abs(z) > band:
            bad.append(k)
    return lines, bad, rows


def annotate(lines, rows):
    """Report lines with the KNOWN_RED reason appended where one applies."""
    out = []
    for line, (tag, k, *_rest) in zip(lines, rows):
        why = KNOWN_RED.get((tag, k))
        out.append(line + (f"   [known red: {why}]" if why else ""))
    return out


def info_row(env, ep, trunc):
    """The logged info keys from the kernel's ep_info row (csrc step_kernel, done)."""
    if env == "descent":
        return {"total_reward": ep[0], "final_altitude": ep[2]}
    if env == "vertical":
        return {"total_reward": ep[0], "total_intrusions": ep[1], "final_altitude": ep[2]}
    if env in ("horizontal", "sector"):
        return {"total_reward": ep[0], "total_intrusions": ep[1], "average_drift": ep[2]}
    if env == "plan":
        return {"total_reward": ep[0], "TimeLimit.truncated": float(trunc)}
    if env == "static":
        return {"waypoint_reached": ep[1], "crashed": ep[2],
                "TimeLimit.truncated": float(trunc)}
    raise KeyError(env)


# ---- MergeEnv-v0: the saturated policy of the DDPG / TD3 logs ------
# tests/golden/merge_logs.npz (extract_merge_logs.py): the last 1,000 episodes of both logs,
# flown by a constant (+-1, +1) action (a circling ownship).  Cases: the reference's
# creation speed (merge_env.py:30 AC_SPD = 100) and the logged revision's (150, as every
# other env of the reference).
MERGE_SAT_KEYS = ("average_drift", "total_intrusions", "total_reward")
MERGE_SAT_HIST = 6                  # intrusions per episode 0..4 and >= 5
_MERGE_SPD = ("the logged intruder stream flies at the Mach cap: the saved SAC model's two "
              "observations put all ten listed intruders at 239.5705 m/s = M0.80 at 10,000 m "
              "(tests/test_last_obs.py), where merge_env.py:30's CAS 100 is 167.5 m/s; the "
              "logged revision created them above CAS 147 (the ac_spd=150 hook is in band)")
_MERGE_DRIFT = ("the ownship's speed over the first steps: it starts at the logged revision's "
                "cap speed, not at CAS 100 (DESIGN.md §5)")
KNOWN_RED.update({
    **{("merge_sat_100", k): _MERGE_SPD for k in ("total_intrusions", "total_reward",
                                                   "intrusion_histogram")},
    ("merge_sat_100", "average_drift"): _MERGE_DRIFT,
})
# Regression bounds on the known-red z of the reference's own creation speed: the
# whitelist above must not hide a further drift of the default config.  Derived from the runs
# they guard (tools/merge_sat_z.py, profiles/r06/merge_sat_z_{oracle,
# device}.json): z against either log over 6 oracle seeds (2,048 envs, tests/test_ref_logs.py's
# size; its seed 11 reads intrusions +3.76 / +3.54) and 8 device seeds (4,096 envs, tests/
# test_gpu_ref_logs.py's size; its seed 7 reads +5.50 / +5.28):
#   intrusions +3.22 .. +5.77 (seed-to-seed sd 0.70 oracle, 0.55 device)
#   reward     -5.65 .. -3.11 (sd 0.71 / 0.55)
#   drift      -4.58 .. -2.92 (sd 0.44 / 0.32)
# Bounds: the measured range widened by two seed-to-seed sd (the larger of the two) each side.
MERGE_SAT_Z_BOUNDS = {("merge_sat_100", "total_intrusions"): (1.8, 7.2),
                      ("merge_sat_100", "total_reward"): (-7.1, -1.7),
                      ("merge_sat_100", "average_drift"): (-5.5, -2.0)}


def merge_logs():
    return dict(np.load(os.path.join(HERE, "golden", "merge_logs.npz")))


def merge_sat_compare(tag, ours: dict, band=BAND_HELDOUT):
    """ours: per-episode average_drift / total_intrusions / total_reward of the saturated
    policy.  Each against both logs: mean z, the drift spread, and the intrusion histogram
    (two-sample chi-square; red below p = 1e-3).  Returns (lines, red statistics)."""
    from scipy.stats import chi2_contingency
    L = merge_logs()
    lines, bad = [], set()
    for alg in ("ddpg", "td3"):
        for k in MERGE_SAT_KEYS:
            x, y = np.asarray(ours[k], np.float64), L[f"{alg}/{k}"]
            se = np.hypot(x.std() / np.sqrt(len(x)), bootstrap_se(y))
            z = (x.mean() - y.mean()) / se
            lines.append(f"{tag} {alg:4s} {k:17s} ours {x.mean():9.4f} sd {x.std():.4f} "
                         f"[{x.min():.3f}, {x.max():.3f}]  log {y.mean():9.4f} sd {y.std():.4f} "
                         f"[{y.min():.3f}, {y.max():.3f}]  z {z:+.2f}")
            if abs(z) > band:
                bad.add(k)
            lo, hi = MERGE_SAT_Z_BOUNDS.get((tag, k), (-np.inf, np.inf))
            if not lo <= z <= hi:
                bad.add(f"{k} (z {z:+.2f} outside its regression bounds [{lo}, {hi}])")
        hx = np.bincount(np.minimum(np.asarray(ours["total_intrusions"], int), MERGE_SAT_HIST - 1),
                         minlength=MERGE_SAT_HIST)
        hy = np.bincount(np.minimum(L[f"{alg}/total_intrusions"].astype(int), MERGE_SAT_HIST - 1),
                         minlength=MERGE_SAT_HIST)
        pval = chi2_contingency(np.stack([hx, hy]))[1]
        lines.append(f"{tag} {alg:4s} P(intrusions = 0..4, >=5) ours {np.round(hx / hx.sum(), 3)} "
                     f"log {np.round(hy / hy.sum(), 3)}  chi2 p {pval:.2g}")
        if pval < 1e-3:
            bad.add("intrusion_histogram")
        ratio = np.std(ours["average_drift"]) / L[f"{alg}/average_drift"].std()
        if not 0.8 < ratio < 1.25:
            bad.add("drift_spread")
    return lines, sorted(bad)
