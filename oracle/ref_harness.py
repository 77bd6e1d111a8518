"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- drive the REFERENCE env code.

Used only by ``tests/golden/make_golden.py`` in the build container (where
``/root/reference`` exists).  It installs in-memory stand-ins for the packages the
reference imports but that are absent offline (gymnasium, pygame, bluesky,
stable_baselines3) and binds ``bluesky`` to a BlueSky-shaped singleton
whose arithmetic is ``oracle.bluesky_subset``.  The reference's own env classes
(MergeEnv, VerticalCREnv, DescentEnv, HorizontalCREnv) and the WindFieldWrapper then run
unmodified and their outputs become the
golden vectors that pin ``oracle.batched``.

Nothing here is imported by the product, and nothing here runs on the GPU box.
"""
from __future__ import annotations

import importlib
import sys
import types

import numpy as np

from . import areas
from . import bluesky_subset as bsx


# --------------------------------------------------------------------------------------
# BlueSky-shaped singleton
# --------------------------------------------------------------------------------------
class _AP:
    def __init__(self, traf):
        self._traf = traf

    @property
    def trk(self):
        """Autopilot.trk (view of the commanded track)."""
        return self._traf.st.ap_trk

    def selaltcmd(self, idx, alt, vspd=None):
        """Autopilot.selaltcmd(idx, alt, vspd)."""
        t = self._traf
        t.selalt[idx] = alt
        t.swvnav[idx] = False
        if vspd:
            t.selvs[idx] = vspd
        else:
            idx_a = np.atleast_1d(idx)
            delalt = alt - t.alt[idx_a]
            opp = np.logical_and(t.selvs[idx_a] * delalt < 0.0, np.abs(t.selvs[idx_a]) > 0.01)
            t.selvs[idx_a[opp]] = 0.0


class Traffic:
    """Subset of bluesky.traffic.Traffic backed by an oracle TrafState of length N."""

    def __init__(self):
        self.wind = bsx.WindField()
        self.reset()
        self.ap = _AP(self)

    # array views used by the env code
    def __getattr__(self, name):
        st = self.__dict__.get("st")
        if st is not None and name in bsx.FIELDS_F64:
            return getattr(st, name)
        raise AttributeError(name)

    def reset(self):
        self.wind.clear()                 # Traffic.reset clears the wind field
        self.st = bsx.TrafState((0,))
        self.id = []
        self.swvnav = np.zeros(0, bool)
        self.routes = []          # per aircraft list of (lat, lon)

    @property
    def ntraf(self):
        return len(self.id)

    def id2idx(self, acid):
        try:
            return self.id.index(acid.upper())
        except ValueError:
            return -1

    def _grow(self, n=1):
        old = self.st
        new = bsx.TrafState((len(self.id) + n,))
        k = len(self.id)
        for f in bsx.FIELDS_F64:
            getattr(new, f)[:k] = getattr(old, f)
        new.swlnav[:k] = old.swlnav
        new.actwp[:k] = old.actwp
        self.st = new
        self.swvnav = np.concatenate([self.swvnav, np.zeros(n, bool)])

    def cre(self, acid, actype="B744", aclat=52.0, aclon=4.0, achdg=None, acalt=0, acspd=0):
        if self.id.count(acid.upper()) > 0:
            return False, acid + " already exists."
        self._grow(1)
        self.id.append(acid.upper())
        self.routes.append([])
        achdg = 0.0 if achdg is None else achdg
        aclon = aclon - 360.0 if aclon > 180.0 else (aclon + 360.0 if aclon < -180.0 else aclon)
        bsx.cre_state(self.st, self.ntraf - 1, aclat, aclon, achdg, acalt, acspd)
        return True

    def creconfs(self, acid, actype, targetidx, dpsi, dcpa, tlosh, dH=None, tlosv=None, spd=None):
        t = self.st
        lat, lon, hdg, acalt, acspd, acvs = bsx.creconfs_params(
            t.lat[targetidx], t.lon[targetidx], t.alt[targetidx], t.trk[targetidx],
            t.gs[targetidx], t.vs[targetidx], dpsi, dcpa, tlosh, dH, tlosv)
        self.cre(acid, actype, lat, lon, hdg, acalt, acspd)
        self.ap.selaltcmd(self.ntraf - 1, t.alt[targetidx], acvs)
        self.st.vs[-1] = acvs

    def delete(self, idx):
        keep = np.ones(self.ntraf, bool)
        keep[idx] = False
        new = bsx.TrafState((int(keep.sum()),))
        for f in bsx.FIELDS_F64:
            setattr(new, f, getattr(self.st, f)[keep])
        new.swlnav = self.st.swlnav[keep]
        new.actwp = self.st.actwp[keep]
        self.st = new
        self.swvnav = self.swvnav[keep]
        self.id = [a for a, k in zip(self.id, keep) if k]
        self.routes = [r for r, k in zip(self.routes, keep) if k]
        return True

    # ---- route / command handlers -----------------------------------------------------
    def addwpt(self, idx, lat, lon):
        r = self.routes[idx]
        r.append((lat, lon))
        if len(r) == 1:                 # first waypoint: direct-to, LNAV on
            self.st.swlnav[idx] = True
            self.st.actwp[idx] = 0

    def update(self, dt):
        if self.ntraf == 0:
            return
        routed = [r for r in self.routes if r]
        if routed:
            ref = routed[0]
            assert all(r == ref for r in routed), "harness supports one shared route"
            rlat = np.array([p[0] for p in ref])
            rlon = np.array([p[1] for p in ref])
            nq = [float(bsx.qdrdist(ref[k][0], ref[k][1], ref[k + 1][0], ref[k + 1][1])[0])
                  for k in range(len(ref) - 1)] + [-999.0]
        else:
            rlat = rlon = np.zeros(0)
            nq = []
        bsx.traffic_update(self.st, dt, rlat, rlon, np.array(nq), self.wind)


class Stack:
    def __init__(self, sim):
        self.queue = []
        self.sim = sim

    def stack(self, cmdline):
        for c in str(cmdline).split(";"):
            c = c.strip()
            if c:
                self.queue.append(c)

    def process(self):
        q, self.queue = self.queue, []
        traf = self.sim.traf
        for c in q:
            w = c.split()
            head = w[0].upper()
            if head == "DT":
                self.sim.simdt = float(w[1])
            elif head in ("FF", "RESO"):
                pass
            elif head == "HDG":
                idx = traf.id2idx(w[1])
                traf.st.ap_trk[idx] = bsx.selhdg_track(traf.st, idx, float(w[2]), traf.wind)
                traf.st.swlnav[idx] = False
            elif head == "SPD":
                idx = traf.id2idx(w[1])
                v = float(w[2])
                traf.st.selspd[idx] = v * bsx.kts if v >= 1.0 else v
            else:
                idx = traf.id2idx(w[0])
                cmd = w[1].upper()
                if idx < 0:
                    raise ValueError(c)
                if cmd in ("ADDWPT", "DEST"):
                    traf.addwpt(idx, float(w[2]), float(w[3]))
                else:
                    raise ValueError("unsupported stack command: " + c)


class Sim:
    def __init__(self):
        self.simdt = 0.05
        self.simt = 0.0
        self.traf = None
        self.stack = None

    def step(self):
        self.stack.process()
        self.simt += self.simdt
        self.traf.update(self.simdt)


def make_bluesky_module():
    bs = types.ModuleType("bluesky")
    bs.__path__ = []
    sim = Sim()
    traf = Traffic()
    stack = Stack(sim)
    sim.traf = traf
    sim.stack = stack
    bs.sim = sim
    bs.traf = traf
    bs.stack = stack
    bs.scr = None

    def init(mode="sim", detached=True, **kw):
        return None
    bs.init = init
    tools = types.ModuleType("bluesky.tools")
    tools.__path__ = []
    geo = types.ModuleType("bluesky.tools.geo")
    for name in ("kwikqdrdist", "kwikdist", "kwikdist_matrix", "kwikqdrdist_matrix",
                 "kwikpos", "qdrdist", "rwgs84"):
        setattr(geo, name, getattr(bsx, name))
    areafilter = areas.AreaFilter()
    af = types.ModuleType("bluesky.tools.areafilter")
    af.defineArea = areafilter.defineArea
    af.deleteArea = areafilter.deleteArea
    af.checkInside = areafilter.checkInside
    tools.areafilter = af
    aero = types.ModuleType("bluesky.tools.aero")
    aero.kts = bsx.kts
    aero.nm = bsx.nm
    aero.ft = bsx.ft
    tools.geo = geo
    tools.aero = aero
    bs.tools = tools
    simulation = types.ModuleType("bluesky.simulation")

    class ScreenIO:
        def __init__(self, *a, **k):
            pass
    simulation.ScreenIO = ScreenIO
    bs.simulation = simulation
    return bs, {"bluesky": bs, "bluesky.tools": tools, "bluesky.tools.geo": geo,
                "bluesky.tools.aero": aero, "bluesky.tools.areafilter": af,
                "bluesky.simulation": simulation}


def _gym_stub():
    gym = types.ModuleType("gymnasium")
    gym.__path__ = []
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float64):
            self.low, self.high, self.shape, self.dtype = low, high, shape or (1,), dtype

    class Dict(dict):
        def __init__(self, d):
            super().__init__(sorted(d.items()))
            self.spaces = dict(self)
    spaces.Box = Box
    spaces.Dict = Dict

    class Env:
        metadata = {}

        def reset(self, seed=None, options=None):
            return None
    gym.Env = Env

    class Wrapper:
        def __init__(self, env):
            self.env = env
            self._obs_space = None

        @property
        def observation_space(self):
            return self._obs_space if self._obs_space is not None else self.env.observation_space

        @observation_space.setter
        def observation_space(self, v):
            self._obs_space = v

        def reset(self, **kw):
            return self.env.reset(**kw)

        def step(self, action):
            return self.env.step(action)

        def __getattr__(self, name):
            return getattr(self.__dict__["env"], name)
    gym.Wrapper = Wrapper
    gym.spaces = spaces
    envs = types.ModuleType("gymnasium.envs")
    envs.__path__ = []
    reg = types.ModuleType("gymnasium.envs.registration")
    reg.register = lambda **kw: None
    envs.registration = reg
    gym.envs = envs
    return {"gymnasium": gym, "gymnasium.spaces": spaces, "gymnasium.envs": envs,
            "gymnasium.envs.registration": reg}


def _misc_stubs():
    pygame = types.ModuleType("pygame")
    sb3 = types.ModuleType("stable_baselines3")
    sb3.__path__ = []
    common = types.ModuleType("stable_baselines3.common")
    common.__path__ = []
    cb = types.ModuleType("stable_baselines3.common.callbacks")

    class BaseCallback:
        def __init__(self, verbose=0):
            pass
    cb.BaseCallback = BaseCallback
    return {"pygame": pygame, "stable_baselines3": sb3, "stable_baselines3.common": common,
            "stable_baselines3.common.callbacks": cb}


def load_reference_envs(reference_root="/root/reference"):
    """Import the reference env modules with the stand-ins installed.  Returns
    (bs_singleton, {'merge': module, 'vertical': module, 'descent': module})."""
    bs, bsmods = make_bluesky_module()
    saved = {}
    mods = {}
    mods.update(bsmods)
    mods.update(_gym_stub())
    mods.update(_misc_stubs())
    for k, v in mods.items():
        saved[k] = sys.modules.get(k)
        sys.modules[k] = v
    if reference_root not in sys.path:
        sys.path.insert(0, reference_root)
    # import env modules directly (bluesky_gym/__init__ would import SB3 callbacks too)
    for k in list(sys.modules):
        if k == "bluesky_gym" or k.startswith("bluesky_gym."):
            del sys.modules[k]
    pkg = types.ModuleType("bluesky_gym")
    pkg.__path__ = [reference_root + "/bluesky_gym"]
    sys.modules["bluesky_gym"] = pkg
    envs_pkg = types.ModuleType("bluesky_gym.envs")
    envs_pkg.__path__ = [reference_root + "/bluesky_gym/envs"]
    sys.modules["bluesky_gym.envs"] = envs_pkg
    wr_pkg = types.ModuleType("bluesky_gym.wrappers")
    wr_pkg.__path__ = [reference_root + "/bluesky_gym/wrappers"]
    sys.modules["bluesky_gym.wrappers"] = wr_pkg
    out = {
        "merge": importlib.import_module("bluesky_gym.envs.merge_env"),
        "vertical": importlib.import_module("bluesky_gym.envs.vertical_cr_env"),
        "descent": importlib.import_module("bluesky_gym.envs.descent_env"),
        "horizontal": importlib.import_module("bluesky_gym.envs.horizontal_cr_env"),
        "static": importlib.import_module("bluesky_gym.envs.static_obstacle_env"),
        "sector": importlib.import_module("bluesky_gym.envs.sector_cr_env"),
        "plan": importlib.import_module("bluesky_gym.envs.plan_waypoint_env"),
        "functions": importlib.import_module("bluesky_gym.envs.common.functions"),
        "wind": importlib.import_module("bluesky_gym.wrappers.wind"),
        "uncertainty": importlib.import_module("bluesky_gym.wrappers.uncertainty"),
    }
    return bs, out
