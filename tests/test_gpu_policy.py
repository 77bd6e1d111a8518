"""GPU checks of the fused SAC actor kernel (bsg_policy_sac, csrc/bsg_policy.hip) against a
plain PyTorch reference of the same op (SB3 SAC Actor: Linear-ReLU 256-256, mu / log_std
heads, log_std clamped to [-20, 2], tanh squash, log-prob with the 1e-6 tanh correction),
evaluated in float64 from the same fp32 weights and inputs.

Tolerances: the kernel's actions are within max(2e-5, 4 x the error of torch's own fp32
forward) of the float64 reference (both round fp32 256-term dot products in different
orders, so their worst rows over a batch differ by small factors; with N(0, 4) inputs far
outside the actors' training range the pre-activations reach ~1e2 and fp32 rounding reaches
a few 1e-5 in either); inputs are seeded; log_prob 2e-3 absolute where 1 - a^2 > 1e-2
(log(1 - a^2) amplifies the action's rounding near +-1, where it is not compared)."""
import os

import numpy as np
import pytest
import torch

from bluesky_gym import _native as nat
from bluesky_gym.policy import SACPolicy

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "sac_actors.npz")
TAGS = ("descent", "vertical", "horizontal", "plan", "static", "sector")
KEYS = ("latent_pi.0.weight", "latent_pi.0.bias", "latent_pi.2.weight", "latent_pi.2.bias",
        "mu.weight", "mu.bias", "log_std.weight", "log_std.bias")


def ref_actor(W, obs, eps, dtype=torch.float64):
    """float64 (or fp32: torch's own forward) restatement of SB3's Actor.forward +
    action_log_prob."""
    w = [torch.as_tensor(W[k], dtype=dtype, device=obs.device) for k in KEYS]
    x = obs.to(dtype)
    h = torch.relu(x @ w[0].T + w[1])
    h = torch.relu(h @ w[2].T + w[3])
    mu = h @ w[4].T + w[5]
    ls = torch.clamp(h @ w[6].T + w[7], -20.0, 2.0)
    e = torch.zeros_like(mu) if eps is None else eps.to(dtype)
    u = mu + ls.exp() * e
    a = torch.tanh(u)
    lp = (-0.5 * e * e - ls - 0.5 * np.log(2 * np.pi)).sum(-1) - torch.log(1 - a * a + 1e-6).sum(-1)
    return a, lp


def check_actions(act, W, obs, eps):
    ra = ref_actor(W, obs, eps)[0]
    terr = (ref_actor(W, obs, eps, torch.float32)[0].double() - ra).abs().max().item()
    err = (act - ra).abs().max().item()
    assert err <= max(2e-5, 4 * terr), (err, terr)


def weights(tag):
    with np.load(GOLD) as z:
        return {k: z[f"{tag}/{k}"] for k in KEYS}


@pytest.mark.parametrize("tag", TAGS)
@pytest.mark.parametrize("E,extra", [(1, 0), (15, 3), (16, 0), (17, 3), (4096, 3)])
def test_policy_matches_torch_reference(tag, E, extra):
    dev = torch.device("cuda", 0)
    W = weights(tag)
    pol = SACPolicy(W, dev)
    O, A = pol.obs_dim, pol.act_dim
    g = torch.Generator(device=dev).manual_seed(E * 7 + O)
    # rows with `extra` trailing columns, as the learner rows [obs | reward | term | trunc]
    rows = torch.randn((E, O + extra), generator=g, device=dev) * 2
    obs = rows[:, :O] if extra else rows
    eps = torch.randn((E, A), generator=g, device=dev)
    for e in (None, eps):
        lp = torch.full((E,), float("nan"), device=dev)
        act = pol(obs, e, log_prob=lp)
        ra, rlp = ref_actor(W, obs, e)
        terr = (ref_actor(W, obs, e, torch.float32)[0].double() - ra).abs().max().item()
        assert act.dtype == torch.float64 and act.shape == (E, A)
        err = (act - ra).abs().max().item()
        assert err <= max(2e-5, 4 * terr), (tag, E, e is None, err, terr)
        print(f"{tag} E={E} eps={e is not None}: kernel {err:.2e}, torch fp32 {terr:.2e}")
        ok = (1 - ra * ra).min(-1).values > 1e-2
        lerr = (lp.double() - rlp)[ok].abs().max().item() if ok.any() else 0.0
        assert lerr <= 2e-3, (tag, E, lerr)
        assert torch.isfinite(lp).all()


def test_policy_shares_live_module_weights_and_replays_in_graph():
    """from_module reads the torch actor's parameters by pointer: an in-place update (what
    the learner's optimizer does) is seen by the next call, also by a captured HIP graph."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import sac_torch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    actor = sac_torch.Actor(4, 1).to(dev)
    actor.load_sb3(np.load(GOLD), "descent")
    pol = SACPolicy.from_module(actor)
    obs = torch.randn((4096, 4), device=dev)
    eps = torch.randn((4096, 1), device=dev)
    out = torch.empty((4096, 1), dtype=torch.float64, device=dev)
    W = {k: getattr_param(actor, k).detach().cpu().numpy() for k in KEYS}
    pol(obs, eps, out=out)
    check_actions(out, W, obs, eps)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        pol(obs, eps, out=out)
    torch.cuda.current_stream(dev).wait_stream(side)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        torch.randn((4096, 1), device=dev, out=eps)
        pol(obs, eps, out=out)
    with torch.no_grad():
        actor.mu.bias.add_(0.25)
        actor.latent[2].weight.mul_(0.9)
    obs.copy_(torch.randn_like(obs))
    gr.replay()
    torch.cuda.synchronize()
    W = {k: getattr_param(actor, k).detach().cpu().numpy() for k in KEYS}
    check_actions(out, W, obs, eps)
    e1 = eps.clone()
    gr.replay()
    torch.cuda.synchronize()
    assert not torch.equal(e1, eps)                       # fresh noise per replay
    check_actions(out, W, obs, eps)


def getattr_param(actor, key):
    m = {"latent_pi.0": actor.latent[0], "latent_pi.2": actor.latent[2], "mu": actor.mu,
         "log_std": actor.log_std}
    mod, attr = key.rsplit(".", 1)
    return getattr(m[mod], attr)


def test_policy_drives_device_batch():
    """The policy writes the action rows bsg_step reads: a Descent batch stepped with
    SACPolicy's deterministic actions equals one stepped with the torch reference's actions
    rounded the same way (the kernel's actions are used as given)."""
    from bluesky_gym import config, core
    dev = torch.device("cuda", 0)
    W = weights("descent")
    pol = SACPolicy(W, dev)
    b = core.DeviceBatch(config.descent_config(), 512, autoreset=nat.AUTORESET_SAME_STEP,
                         compute_cd=False, seed=5)
    b.reset()
    act = torch.empty((512, 1), dtype=torch.float64, device=dev)
    steps = 0
    for _ in range(40):
        pol(b.obs, None, out=act)
        check_actions(act, W, b.obs, None)
        b.step(act)
        steps += 1
    torch.cuda.synchronize()
    assert torch.isfinite(b.obs).all() and steps == 40


def test_policy_rejects_bad_shapes():
    dev = torch.device("cuda", 0)
    W = weights("descent")
    pol = SACPolicy(W, dev)
    with pytest.raises(ValueError):
        pol(torch.zeros((8, 4), dtype=torch.float64, device=dev))
    with pytest.raises(ValueError):
        pol(torch.zeros((8, 4), device=dev), torch.zeros((8, 2), device=dev))
    bad = dict(W)
    bad["latent_pi.2.weight"] = np.zeros((128, 256), np.float32)
    with pytest.raises(ValueError):
        SACPolicy(bad, dev)
    pol(torch.zeros((0, 4), device=dev))                 # empty batch is a no-op
    p2 = SACPolicy.from_npz(GOLD, "descent", "cuda")     # an index-less device string
    assert p2(torch.zeros((8, 4), device=dev)).shape == (8, 1)
