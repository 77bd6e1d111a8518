"""The device sim layer against the reference's own simulator, value by value: the saved
models' observations (tests/golden/last_obs.npz; tests/last_obs_pins.py) on
the HIP path -- the same pins tests/test_last_obs.py holds the oracle to.  The device's
fp64 state is compared where it exists, its fp32 observation rows otherwise (tolerance:
the fixture's print precision plus fp32 rounding of the row)."""
import numpy as np
import pytest
import torch

import last_obs_pins as lp
from oracle import bluesky_subset as bsx

pytestmark = pytest.mark.gpu

SAVED_MERGE_AIRSPEED = 239.5705319
E = 64


def _batch(cfg, **kw):
    from bluesky_gym import core
    b = core.DeviceBatch(cfg, E, seed=4, **kw)
    b.reset()
    return b


def test_device_merge_ownship_holds_the_saved_airspeed():
    """SPD +20 m/s every step: the ownship's fp64 TAS settles at the Mach cap the saved Merge
    states record (239.5705319 m/s), and so does the fp32 airspeed obs."""
    from bluesky_gym import config
    from bluesky_gym.obs_layout import ObsLayout
    b = _batch(config.merge_config(num_ac=20))
    act = torch.tensor([[0.0, 1.0]], dtype=torch.float64, device=b.device).expand(E, 2).contiguous()
    for _ in range(8):
        b.step(act)
    torch.cuda.synchronize()
    cap = float(bsx.vmach2tas(bsx.MMO, 10000.0))
    tas0 = b.state["tas"][:, 0].cpu().numpy()
    assert np.all(np.abs(tas0 - cap) <= 1e-9), tas0
    lay = ObsLayout(config.merge_config(num_ac=20).kind, 20, 5)
    airspeed = b.obs[:, lay.slices["airspeed"]].cpu().numpy()[:, 0]
    assert np.all(np.abs(airspeed - SAVED_MERGE_AIRSPEED) <= 2e-5)


@pytest.mark.parametrize("ac_spd", [100, 150])
def test_device_merge_intruder_speed(ac_spd):
    """The intruders' speed in the saved Merge states is the Mach cap (the logged revision's
    creation CAS 150); merge_env.py:30's CAS 100 gives 167.5 m/s.  The device holds both."""
    from bluesky_gym import config
    b = _batch(config.merge_config(num_ac=20, ac_spd=ac_spd))
    zero = torch.zeros((E, 2), dtype=torch.float64, device=b.device)
    for _ in range(4):
        b.step(zero)
    torch.cuda.synchronize()
    want = float(bsx.vmach2tas(bsx.MMO, 10000.0)) if ac_spd == 150 else float(bsx.vcas2tas(100.0, 10000.0))
    tas = b.state["tas"][:, 1:].cpu().numpy()
    assert np.all(np.abs(tas - want) <= 1e-9)
    if ac_spd == 150:
        speeds, _h, steady, _s = lp.merge_intruder_speeds(lp.load())
        assert np.all(np.abs(speeds[:, steady] - float(tas[0, 0])) < 1e-4)


@pytest.mark.parametrize("env", ["DescentEnv-v0", "VerticalCREnv-v0"])
def test_device_reproduces_the_saved_vertical_transition(env):
    """Every env's ownship is put in the state of the SAC model's first observation
    (lp.ownship_start) and stepped once under the action its second observation holds; the
    kernel's altitude, vz and runway_distance obs must be the saved second observation."""
    from bluesky_gym import config
    from bluesky_gym.obs_layout import ObsLayout
    cfg = config.descent_config() if env == "DescentEnv-v0" else config.vertical_config()
    b = _batch(cfg, compute_cd=False)
    L = lp.load()
    t0 = lp.vertical_ownship(L, env, "SAC", lp.BEFORE)
    s = lp.ownship_start(bsx, t0)
    st = b.state
    for k, v in (("lat", s["lat"]), ("lon", s["lon"]), ("alt", s["alt"]), ("hdg", s["hdg"]),
                 ("tas", s["tas"]), ("cas", s["cas"]), ("vs", s["vs"]), ("ax", 0.0),
                 ("ap_trk", s["hdg"]), ("selspd", s["selspd"])):
        st[k][:, 0] = v
    b.envs["target_alt"][:] = t0["tgt"]
    b.envs["step_count"][:] = 8
    b.invalidate_caches()
    a = lp.implied_action(L, env, "SAC")
    b.step(torch.full((E, 1), a, dtype=torch.float64, device=b.device))
    torch.cuda.synchronize()
    assert not b.terminated.any() and not b.truncated.any()
    lay = ObsLayout(cfg.kind, cfg.num_ac, cfg.num_ac_state)
    got = b.obs.cpu().numpy().astype(np.float64)
    want = lp.obs(L, env, "SAC", lp.AFTER)
    for k in ("altitude", "vz", "runway_distance", "target_altitude"):
        g = got[:, lay.slices[k]][:, 0]
        assert np.all(np.abs(g - want[k][0]) <= 1e-7 + 1e-7 * abs(want[k][0])), (k, g[:3], want[k])
    alt = st["alt"][:, 0].cpu().numpy()
    assert np.all(np.abs(alt - (lp.ALT_MEAN + lp.ALT_STD * want["altitude"][0])) <= 2e-5)


def test_device_phase_gd_cap_is_the_saved_horizontal_speed():
    """HorizontalCREnv's aircraft (created at alt 0, phase GD) fly the cap the saved Horizontal
    states record for every aircraft: 89.000 m/s."""
    from bluesky_gym import config
    b = _batch(config.horizontal_config(), compute_cd=False)
    zero = torch.zeros((E, 1), dtype=torch.float64, device=b.device)
    for _ in range(8):
        b.step(zero)
    torch.cuda.synchronize()
    # envs at least 7 steps (35 s) into their episode: CAS 150 -> 89 at axmax 2 takes 31 s
    live = b.envs["step_count"].cpu().numpy() >= 7
    tas = b.state["tas"].cpu().numpy()[live]
    assert live.sum() > E // 2 and np.all(np.abs(tas - 89.0) <= 5e-8)
