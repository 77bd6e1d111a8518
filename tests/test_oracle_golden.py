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
