"""The reference's saved SAC actors and the tails of its SAC training logs, as a
distributional pin of the BlueSky sim layer (parity of the simulator arithmetic is
otherwise unpinned: bluesky-simulator is not vendored).

Fixture: tests/golden/sac_actors.npz (tests/golden/extract_sac_actors.py): per env the
SB3 SAC actor (stable-baselines3 2.2.1 `Actor`: Linear-ReLU-Linear-ReLU 256/256, `mu`,
`log_std` clamped to [-20, 2], action = tanh(mu + std * eps) while training) and the
last 1,000 episodes the training run logged (scripts/common/logger.py:15-36).

The logged episodes were produced by the policy while it was still being trained; the
saved actor is the final one, so the comparison is statistical: every compared mean must
lie within BAND standard errors of the log's (bootstrap SE of the log, normal SE of the
rollout, combined in quadrature).
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BAND = 4.0

# info keys compared per env (plus the episode length)
LOG_KEYS = {
    "descent": ("total_reward", "final_altitude"),
    "vertical": ("total_reward", "total_intrusions", "final_altitude"),
    "horizontal": ("total_reward", "total_intrusions", "average_drift"),
    "plan": ("total_reward", "TimeLimit.truncated"),
}


def load():
    return dict(np.load(os.path.join(HERE, "golden", "sac_actors.npz")))


def actor_np(W, tag, obs, rng=None):
    """SAC actor on float32 observations (SB3 feeds the policy float32); float64 math.
    rng None = the deterministic action tanh(mu)."""
    g = lambda k: W[f"{tag}/{k}"].astype(np.float64)  # noqa: E731
    x = np.asarray(obs, np.float32).astype(np.float64)
    h = np.maximum(x @ g("latent_pi.0.weight").T + g("latent_pi.0.bias"), 0.0)
    h = np.maximum(h @ g("latent_pi.2.weight").T + g("latent_pi.2.bias"), 0.0)
    mu = h @ g("mu.weight").T + g("mu.bias")
    if rng is None:
        return np.tanh(mu)
    ls = np.clip(h @ g("log_std.weight").T + g("log_std.bias"), -20.0, 2.0)
    return np.tanh(mu + np.exp(ls) * rng.standard_normal(mu.shape))


class TorchActor:
    """The same actor as torch fp32 modules on a device (the learner-side forward)."""

    def __init__(self, W, tag, device):
        import torch
        t = lambda k: torch.as_tensor(W[f"{tag}/{k}"], device=device)  # noqa: E731
        self.w = [t(k) for k in ("latent_pi.0.weight", "latent_pi.0.bias", "latent_pi.2.weight",
                                 "latent_pi.2.bias", "mu.weight", "mu.bias", "log_std.weight",
                                 "log_std.bias")]
        self.torch = torch

    def __call__(self, obs, gen=None):
        F = self.torch.nn.functional
        w0, b0, w2, b2, wm, bm, ws, bs = self.w
        h = F.relu(F.linear(obs, w0, b0))
        h = F.relu(F.linear(h, w2, b2))
        mu = F.linear(h, wm, bm)
        if gen is None:
            return self.torch.tanh(mu)
        ls = self.torch.clamp(F.linear(h, ws, bs), -20.0, 2.0)
        eps = self.torch.randn(mu.shape, device=mu.device, generator=gen)
        return self.torch.tanh(mu + self.torch.exp(ls) * eps)


def log_stats(W, tag):
    return {k: W[f"{tag}/log/{k}"] for k in LOG_KEYS[tag] + ("length",)}


def bootstrap_se(x, reps=2000, seed=0):
    x = np.asarray(x, np.float64)
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, len(x), (reps, len(x)))
    return float(x[idx].mean(axis=1).std())


def compare(W, tag, ours: dict, band=BAND):
    """Per statistic: (ours mean, log mean, z = difference / combined SE).  Returns the
    report lines and the statistics outside the band."""
    log = log_stats(W, tag)
    lines, bad = [], []
    for k, lv in log.items():
        ov = np.asarray(ours[k], np.float64)
        se = np.hypot(bootstrap_se(lv), ov.std() / np.sqrt(len(ov)))
        z = (ov.mean() - lv.mean()) / max(se, 1e-12)
        lines.append(f"{tag:10s} {k:20s} ours {ov.mean():10.4f} (n={len(ov)})  "
                     f"log {lv.mean():10.4f}  z {z:+.2f}")
        if abs(z) > band:
            bad.append(k)
    return lines, bad


def info_row(tag, ep, trunc):
    """The logged info keys from the kernel's ep_info row (csrc step_kernel, done)."""
    if tag == "descent":
        return {"total_reward": ep[0], "final_altitude": ep[2]}
    if tag == "vertical":
        return {"total_reward": ep[0], "total_intrusions": ep[1], "final_altitude": ep[2]}
    if tag == "horizontal":
        return {"total_reward": ep[0], "total_intrusions": ep[1], "average_drift": ep[2]}
    if tag == "plan":
        return {"total_reward": ep[0], "TimeLimit.truncated": float(trunc)}
    raise KeyError(tag)
