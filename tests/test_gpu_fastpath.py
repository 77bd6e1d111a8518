"""Specialised substep paths (csrc/bsg_kernels.hip vert_own_fast: the Vertical / Descent
ownship climbing or descending between its altitude commands) against the general
substep() they specialise: a batch created with BSG_NO_FASTPATH=1 runs substep() only.
Every output and every state buffer must be bit-identical step by step, through
autoresets (both conventions), crashes (alt <= 0), the kept aircraft of Descent and the
speculation's fallbacks (ground phase near the runway, a target altitude reached)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

OUTS = ("obs", "reward", "terminated", "truncated", "intr_mask", "conf_mask", "los_mask",
        "tcpamax", "min_sep", "ep_info", "final_obs")


def _batch(cfg, E, general, autoreset, cd):
    from bluesky_gym import core
    old = os.environ.get("BSG_NO_FASTPATH")
    os.environ["BSG_NO_FASTPATH"] = "1" if general else "0"
    try:
        return core.DeviceBatch(cfg, E, autoreset=autoreset, compute_cd=cd, seed=21)
    finally:
        if old is None:
            os.environ.pop("BSG_NO_FASTPATH")
        else:
            os.environ["BSG_NO_FASTPATH"] = old


def _snap(b):
    d = {k: getattr(b, k).clone() for k in OUTS if getattr(b, k, None) is not None}
    d.update({"state." + k: v.clone() for k, v in b.state.items()})
    d.update({"env." + k: v.clone() for k, v in b.envs.items()})
    return d


def _same(x, y, t):
    for k in x:
        a, b = x[k], y[k]
        if a.dtype.is_floating_point:
            a = a.view(torch.int64 if a.element_size() == 8 else torch.int32)
            b = b.view(torch.int64 if b.element_size() == 8 else torch.int32)
        if not torch.equal(a, b):
            raise AssertionError(f"step {t}: {k} differs at {torch.nonzero(a != b)[:4].tolist()}")


@pytest.mark.parametrize("kind,autoreset", [("descent", 1), ("descent", 2), ("vertical", 1),
                                            ("vertical", 2), ("descent25", 2)])
def test_vertical_ownship_fastpath_bit_identical(kind, autoreset):
    """descent25: 25 substeps per step -- not the 3 x 10 the seven-wave pipeline takes, so the
    one-wave blocks (two of 10, then five single substeps) run instead."""
    from bluesky_gym import config
    cfg = (config.descent_config(max_episode_steps=60) if kind == "descent"
           else config.descent_config(action_frequency=25, max_episode_steps=60) if kind == "descent25"
           else config.vertical_config(num_intruders=31, max_episode_steps=60))
    E = 1024 if kind.startswith("descent") else 256
    cd = kind == "vertical"
    gen, fast = _batch(cfg, E, True, autoreset, cd), _batch(cfg, E, False, autoreset, cd)
    g = torch.Generator(device="cuda").manual_seed(4)
    gen.reset()
    fast.reset()
    ends = 0
    for t in range(150):
        # mostly dives and climbs at the command limits (the binding vsmax and the ground
        # phase included), some small commands (|selvs| <= 0.1: the default 1500 fpm)
        a = torch.rand((E, 1), dtype=torch.float64, device="cuda", generator=g) * 2.4 - 1.2
        a = a.clamp(-1, 1)
        a[::7] *= 0.005
        gen.step(a)
        fast.step(a)
        _same(_snap(gen), _snap(fast), t)
        ends += int((gen.terminated | gen.truncated).sum())
    assert ends >= E                                     # episodes ended inside the window


@pytest.mark.parametrize("memo", [True, False])
def test_merge_ownship_fastpath_bit_identical(memo):
    """merge_own_fast (the lookahead's main waves: level HDG/SPD ownships) against
    substep(): both batches run the lookahead; one with BSG_NO_FASTPATH=1.  Turns both
    ways, speed commands into the envelope clamps, NEXT_STEP autoresets (a spawned ownship's
    first step runs substep(): its heading is bearing - 180), and with the memo cache off."""
    from bluesky_gym import config, core
    cfg = config.merge_config(num_ac=32, max_episode_steps=40)
    E = 512
    bs = []
    for general in (True, False):
        old = os.environ.get("BSG_NO_FASTPATH")
        os.environ["BSG_NO_FASTPATH"] = "1" if general else "0"
        try:
            bs.append(core.DeviceBatch(cfg, E, compute_cd=True, seed=8, learner=True,
                                       memo_cache=memo, lookahead=True))
        finally:
            if old is None:
                os.environ.pop("BSG_NO_FASTPATH")
            else:
                os.environ["BSG_NO_FASTPATH"] = old
    gen, fast = bs
    assert gen.lookahead and fast.lookahead
    g = torch.Generator(device="cuda").manual_seed(6)
    gen.reset()
    fast.reset()
    ends = 0
    for t in range(120):
        a = torch.rand((E, 2), dtype=torch.float64, device="cuda", generator=g) * 2.4 - 1.2
        a = a.clamp(-1, 1)
        a[::5] = 0.0                                     # straight and steady: no turn, no speed change
        gen.step(a)
        fast.step(a)
        _same(_snap(gen), _snap(fast), t)
        ends += int((gen.terminated | gen.truncated).sum())
    assert ends >= 2 * E


def test_descent_fastpath_edges_bit_identical():
    """vert_own_fast's blocks (three passes per 10 substeps) at the edges its chains handle
    by a wave-uniform slow variant or a cached branch: a dive reversed just above the ground
    (the altitude overshoots below sea level: the libm pow of vatmos), a climber crossing
    11 km (the stratosphere factor), an aircraft on the ground under a descend command (the
    on-target limits), mixed in every wave with ordinary lanes -- against substep() alone."""
    from bluesky_gym import config
    cfg = config.descent_config(max_episode_steps=300)
    E = 256
    gen, fast = _batch(cfg, E, True, 2, False), _batch(cfg, E, False, 2, False)
    gen.reset()
    fast.reset()
    lane = torch.arange(E, device="cuda") % 4
    for b in (gen, fast):
        st = b.state
        st["alt"][:, 0] = torch.where(lane == 0, 22.0, torch.where(lane == 1, 10950.0,
                                      torch.where(lane == 2, 0.0, st["alt"][:, 0])))
        st["vs"][:, 0] = torch.where(lane == 0, -12.0, torch.where(lane == 1, 12.0,
                                     torch.where(lane == 2, 0.0, st["vs"][:, 0])))
        st["selalt"][:, 0] = torch.where(lane == 1, 1e6, torch.where(lane == 3, st["selalt"][:, 0], 0.0))
        b.invalidate_caches()
    g = torch.Generator(device="cuda").manual_seed(9)
    for t in range(6):
        a = torch.rand((E, 1), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        a[lane == 0] = 1.0 if t == 0 else a[lane == 0]       # reverse the dive at 22 m
        a[lane == 1] = 1.0                                    # keep climbing through 11 km
        a[lane == 2] = -1.0                                   # stay on the ground
        gen.step(a)
        fast.step(a)
        _same(_snap(gen), _snap(fast), t)
    alt = fast.state["alt"][:, 0]
    assert bool((alt[lane == 1] > 11000.0).all())
