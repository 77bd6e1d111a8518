"""The lookahead (bsg_set_lookahead; csrc/bsg_kernels.hip lookahead_role): extra
workgroups propagate the intruders one RL step ahead (Merge's LNAV flight and Vertical's
creconfs straight lines do not depend on the ownship or the action, merge_env.py:155-157,
vertical_cr_env.py:183-200) and the next step consumes that state.
It must be invisible: every output and every state buffer bit-identical to the inline
path, step by step, through NEXT_STEP autoresets, explicit masked resets, host-supplied
spawn rows, a direct state write (invalidate_caches) and turning it off and on."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

OUTS = ("obs", "reward", "terminated", "truncated", "topk", "intr_mask", "conf_mask",
        "los_mask", "tcpamax", "min_sep", "ep_info", "learner")


def _batch(E, N, la, seed=5, maxep=20, kind="merge"):
    from bluesky_gym import config, core
    cfg = (config.merge_config(num_ac=N, max_episode_steps=maxep) if kind == "merge" else
           config.vertical_config(num_intruders=N - 1, max_episode_steps=maxep))
    return core.DeviceBatch(cfg, E, compute_cd=True, seed=seed, learner=True, lookahead=la)


def _snap(b):
    d = {k: getattr(b, k).clone() for k in OUTS if getattr(b, k) is not None}
    for k, v in b.state.items():
        d["state." + k] = v.clone()
    for k, v in b.envs.items():
        d["env." + k] = v.clone()
    return d


def _same(x, y, t):
    for k in x:
        a, b = x[k], y[k]
        if a.dtype.is_floating_point:
            a = a.view(torch.int64 if a.element_size() == 8 else torch.int32)
            b = b.view(torch.int64 if b.element_size() == 8 else torch.int32)
        if not torch.equal(a, b):
            idx = torch.nonzero(a != b)[:4].tolist()
            raise AssertionError(f"step {t}: {k} differs at {idx}")


@pytest.mark.parametrize("kind,E,N", [("merge", 512, 32), ("merge", 100, 20), ("merge", 256, 16),
                                      ("vertical", 512, 32), ("vertical", 100, 6)])
def test_lookahead_bit_identical_to_inline(kind, E, N):
    """Vertical's main waves also run the ownship's fast loop (vert_own_fast) under the
    lookahead: compared here with the inline general substep()."""
    ref, la = _batch(E, N, False, kind=kind), _batch(E, N, True, kind=kind)
    assert la.lookahead and not ref.lookahead
    g = torch.Generator(device="cuda").manual_seed(2)
    ref.reset()
    la.reset()
    _same(_snap(ref), _snap(la), -1)
    dones = 0
    for t in range(90):
        a = torch.rand((E, la.act_dim), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        ref.step(a)
        la.step(a)
        _same(_snap(ref), _snap(la), t)
        dones += int((ref.terminated | ref.truncated).sum())
        if t == 40:                    # an explicit masked reset (Env.reset of some envs)
            m = (torch.arange(E, device="cuda") % 3 == 0).to(torch.uint8)
            ref.reset(m)
            la.reset(m)
            _same(_snap(ref), _snap(la), t)
        if t == 60:                    # a direct state write + the documented re-arm
            for b in (ref, la):
                b.state["lat"][:, 3] += 1e-3
                b.invalidate_caches()
    torch.cuda.synchronize()
    assert dones >= E * 3                               # autoresets in the window


@pytest.mark.parametrize("kind", ["merge", "vertical"])
def test_lookahead_with_host_spawn_rows_and_toggle(kind):
    """Parity mode (host spawn rows for the NEXT_STEP resets) and switching the lookahead
    off and on mid-run keep the outputs bit-identical."""
    import ctypes as C
    from bluesky_gym import _native as nat
    from bluesky_gym.spawn import merge_spawn, vertical_spawn
    E, N = 128, 32
    ref, la = _batch(E, N, False, seed=9, kind=kind), _batch(E, N, True, seed=9, kind=kind)
    rs = np.random.RandomState(4)
    g = torch.Generator(device="cuda").manual_seed(8)

    def rows():
        one = (lambda: merge_spawn(N, rs)) if kind == "merge" else (lambda: vertical_spawn(N - 1, rs))
        return torch.from_numpy(np.stack([one() for _ in range(E)])).cuda()

    sp = rows()
    ref.reset(spawn=sp)
    la.reset(spawn=sp)
    for t in range(70):
        a = torch.rand((E, la.act_dim), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        sp = rows()
        ref.step(a, spawn=sp)
        la.step(a, spawn=sp)
        _same(_snap(ref), _snap(la), t)
        if t == 25:
            nat.check(la.lib.bsg_set_lookahead(la._ctx, None, 0), "off")
        if t == 45:
            nat.check(la.lib.bsg_set_lookahead(la._ctx, C.c_void_p(la._la_buf.data_ptr()),
                                               la._la_buf.numel() * 8), "on")


def test_lookahead_refused_where_unsupported():
    from bluesky_gym import _native as nat, config, core
    with pytest.raises(nat.BsgError):
        core.DeviceBatch(config.descent_config(), 64, lookahead=True)
    with pytest.raises(nat.BsgError):
        core.DeviceBatch(config.vertical_config(), 64, autoreset=nat.AUTORESET_SAME_STEP,
                         lookahead=True)
    with pytest.raises(nat.BsgError):
        core.DeviceBatch(config.merge_config(num_ac=16), 64,
                         autoreset=nat.AUTORESET_SAME_STEP, lookahead=True)
    b = core.DeviceBatch(config.merge_config(num_ac=16), 64)     # auto: on for Merge shards
    assert b.lookahead
