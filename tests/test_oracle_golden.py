"""Pin the CPU oracle (oracle/batched.py) to the REFERENCE env code.

The golden vectors were produced by running the reference's own merge_env.py,
vertical_cr_env.py and descent_env.py (tests/golden/make_golden.py).  The batched
oracle must reproduce them bit for bit for observations, rewards, terminations,
top-K intruder indices, intrusion masks and aircraft state; the info field
``average_drift`` differs only by summation order (np.mean pairwise vs running sum).
"""
import numpy as np
import pytest

import oracle_replay as rp
from oracle import bluesky_subset as bsx
from oracle import batched as ob

GOLD = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(f"{GOLD}/{name}.npz"))


def test_known_answers_functions():
    k = load("functions_known")
    lat, lon = bsx.get_point_at_distance(52.36239301495972, 4.713195734579777, 200, 0)
    assert (lat, lon) == tuple(k["fix"])
    assert (float(lat), float(lon)) == (54.16103622679719, 4.713195734579777)
    got = [float(bsx.bound_angle_positive_negative_180(a)) for a in k["bound_in"]]
    assert got == k["bound"].tolist()
    assert got[:2] == [-170.0, -180.0]          # single wrap only (functions.py:17-22)
    d = bsx.kwikdist(ob.FIX_LAT, ob.FIX_LON, ob.RWY_LAT, ob.RWY_LON)
    assert float(d) == 107.99136069114495        # SURVEY §4 known answer


@pytest.mark.parametrize("name", ["merge_N8", "merge_N16", "merge_N20", "merge_N32"])
def test_merge_oracle_matches_reference(name):
    g = load(name)
    r = rp.replay_merge(g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    for k in ("obs", "reward", "state"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    assert np.array_equal(r["truncated"][m].astype(np.int8), g["truncated"][m])
    assert np.array_equal(r["topk"][m], g["topk"][m])
    assert np.array_equal(r["intr"][m], g["intr"][m])
    ri, gi = r["info"][m], g["info"][m]
    for c in (0, 1, 3):
        assert np.array_equal(ri[:, c], gi[:, c])
    np.testing.assert_allclose(ri[:, 2], gi[:, 2], rtol=1e-14, atol=0)   # average_drift


def _nonterminal(g):
    m = rp.step_mask(g)
    return m & (g["terminated"] == 0)


@pytest.mark.parametrize("name", ["vertical_N6", "vertical_N32"])
def test_vertical_oracle_matches_reference(name):
    g = load(name)
    r = rp.replay_vertical(g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    for k in ("obs", "reward", "info"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    nt = _nonterminal(g)
    assert np.array_equal(r["state"][nt], g["state"][nt])
    assert np.array_equal(r["intr"][nt], g["intr"][nt])


def test_descent_oracle_matches_reference():
    g = load("descent")
    r = rp.replay_descent(g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    for k in ("obs", "reward", "info"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    nt = _nonterminal(g)
    assert np.array_equal(r["state"][nt], g["state"][nt])


@pytest.mark.parametrize("name", ["horizontal_N6", "horizontal_N16"])
def test_horizontal_oracle_matches_reference(name):
    g = load(name)
    r = rp.replay_horizontal(g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    assert np.array_equal(r["wpt"], g["wpt"])
    for k in ("obs", "reward"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    ri, gi = r["info"][m], g["info"][m]
    for c in (0, 1):
        assert np.array_equal(ri[:, c], gi[:, c])
    np.testing.assert_allclose(ri[:, 2], gi[:, 2], rtol=1e-14, atol=0)   # average_drift
    nt = _nonterminal(g)
    assert np.array_equal(r["state"][nt], g["state"][nt])
    assert np.array_equal(r["intr"][nt], g["intr"][nt])


@pytest.mark.parametrize("name", ["plan", "plan_long", "plan_greedy", "descent_keep"])
def test_kept_aircraft_oracle_matches_reference(name):
    """One env over consecutive episodes: a truncated episode's aircraft carries into the
    next reset (descent_env.py:173, plan_waypoint_env.py:164 cre refused), a terminated
    one is deleted and re-created (descent_env.py:201-204, plan_waypoint_env.py:189-193)."""
    g = load(name)
    r = rp.replay_descent_keep(g) if name == "descent_keep" else rp.replay_plan(g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    if "wpt" in g:
        assert np.array_equal(r["wpt"], g["wpt"])
    for k in ("obs", "reward", "info"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m], g["terminated"][m])
    assert np.array_equal(r["truncated"][m], g["truncated"][m])
    nt = _nonterminal(g)
    assert np.array_equal(r["state"][nt], g["state"][nt])
    # the quirk is exercised: some episode starts from a kept (moved) aircraft
    ends = g["length"] - 1
    kept = [ep for ep in range(1, len(ends)) if g["truncated"][ep - 1, ends[ep - 1]]]
    assert kept


def _eq_obs(r, g, m):
    """Equal observations; the NaN wind keys of a terminal step (the reference wrapper
    raises there, tests/golden/make_golden.py:_step) are excluded."""
    a, b = r["obs"][m], g["obs"][m]
    fin = np.isfinite(b)
    assert np.array_equal(a[fin], b[fin])
    assert (~fin).sum() <= 2 * int(g["terminated"].sum())


@pytest.mark.parametrize("name", ["wind_merge_N16", "wind_vertical_N6", "wind_descent",
                                  "wind_horizontal_N6"])
def test_wind_wrapper_oracle_matches_reference(name):
    """WindFieldWrapper(augment_obs=True) around each env (wrappers/wind.py)."""
    g = load(name)
    kind = name.split("_")[1]
    r = {"merge": rp.replay_merge, "vertical": rp.replay_vertical, "descent": rp.replay_descent,
         "horizontal": rp.replay_horizontal}[kind](g)
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    _eq_obs(r, g, m)
    assert np.array_equal(r["reward"][m], g["reward"][m])
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    nt = _nonterminal(g)
    assert np.array_equal(r["state"][nt], g["state"][nt])


def test_wind_field_interpolation_properties():
    f = bsx.WindField()
    assert f.getdata(52.0, 4.0, 1000.0) == (0.0, 0.0) or f.winddim == 0
    f.addpointvne(52.0, 4.0, np.array([[-12.0]]), np.array([[8.0]]))
    assert f.winddim == 1
    vn, ve = f.getdata(np.array([50.0, 55.0]), np.array([3.0, 9.0]), np.array([0.0, 9000.0]))
    assert np.all(vn == -12.0) and np.all(ve == 8.0)
    g = bsx.WindField()
    g.addpointvne(np.array([51.9, 52.1]), np.array([4.0, 4.0]), np.array([[10.0, 20.0]]),
                  np.array([[0.0, 0.0]]))
    assert g.winddim == 2
    vn, _ = g.getdata(np.array([51.9, 52.0, 52.1]), np.array([4.0, 4.0, 4.0]), 0.0)
    assert abs(vn[0] - 10.0) < 1e-9 and abs(vn[2] - 20.0) < 1e-9 and abs(vn[1] - 15.0) < 1e-6
    h = bsx.WindField()
    h.addpointvne(52.0, 4.0, np.array([[0.0], [30.0]]), np.array([[0.0], [0.0]]),
                  np.array([0.0, 3000.0]))
    assert h.winddim == 3
    # profiles are sampled on the fixed 100 ft axis: exact at axis levels, linear between
    lv = 50 * 100 * 0.3048
    vn, _ = h.getdata(52.0, 4.0, np.array([0.0, lv, lv + 0.5 * 30.48, 3048.0, 20000.0]))
    np.testing.assert_allclose(vn, [0.0, 15.24, 15.24 + 0.5 * 0.3048, 30.0, 30.0], atol=1e-9)


def test_static_oracle_matches_reference():
    """StaticObstacleEnv: geometry built from the host spawn rows equals the reference's,
    and obs / reward / done / info / state replay bit for bit (per-substep reward with the
    previous observation's waypoint distance and drift, static_obstacle_env.py:132-150)."""
    g = load("static")
    r = rp.replay_static(g)
    geo = r["geo"]
    assert np.array_equal(geo["clat"], g["clat"]) and np.array_equal(geo["clon"], g["clon"])
    assert np.array_equal(geo["R"], g["R"]) and np.array_equal(geo["wpt"], g["wpt"])
    for e in range(len(g["length"])):
        for o in range(len(geo["polys"][e])):
            n = int(g["nvert"][e, o])
            assert np.array_equal(geo["polys"][e][o][0], g["poly_lat"][e, o, :n])
            assert np.array_equal(geo["polys"][e][o][1], g["poly_lon"][e, o, :n])
    m = rp.step_mask(g)
    assert np.array_equal(r["obs0"], g["obs0"])
    for k in ("obs", "reward", "state"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    ri, gi = r["info"][m], g["info"][m]
    for c in (0, 1, 2):
        assert np.array_equal(ri[:, c], gi[:, c])
    np.testing.assert_allclose(ri[:, 3], gi[:, 3], rtol=1e-14, atol=0)


def test_sector_oracle_matches_reference():
    g = load("sector_N32")
    r = rp.replay_sector(g)
    m = rp.step_mask(g)
    assert np.array_equal(g["spawn"][:, 0].astype(int), g["num_ac_ep"])
    assert np.array_equal(r["obs0"], g["obs0"])
    for k in ("obs", "reward", "state"):
        assert np.array_equal(r[k][m], g[k][m]), k
    assert np.array_equal(r["terminated"][m].astype(np.int8), g["terminated"][m])
    assert np.array_equal(r["truncated"][m].astype(np.int8), g["truncated"][m])
    assert np.array_equal(r["intr"][m], g["intr"][m])
    ri, gi = r["info"][m], g["info"][m]
    for c in (0, 1):
        assert np.array_equal(ri[:, c], gi[:, c])
    np.testing.assert_allclose(ri[:, 2], gi[:, 2], rtol=1e-14, atol=0)


def test_merge_distribution_sanity():
    """Random-policy Merge episodes land in the published untrained-policy band
    (~1.3-1.5 intrusions, ~-9 return, average drift ~1.5 rad)."""
    o = ob.MergeOracle(64, num_ac=20, autoreset=ob.AUTORESET_NONE, compute_cd=False, seed=7)
    o.reset()
    rng = np.random.default_rng(0)
    alive = np.ones(64, bool)
    for t in range(50):
        r = o.step(rng.uniform(-1, 1, (64, 2)))
        alive &= ~(r["terminated"] | r["truncated"])
    inf = o.info()
    assert 0.3 < inf["total_intrusions"].mean() < 4.0
    assert 0.8 < np.nanmean(inf["average_drift"]) < 2.2
