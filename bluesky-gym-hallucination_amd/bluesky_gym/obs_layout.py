"""Observation layouts: the reference observation_space keys, their sizes and the
flat (sorted-key) offsets the HIP kernel writes.

merge_env.py:59-74, vertical_cr_env.py:67-83, descent_env.py:53-60,
horizontal_cr_env.py:49-60, static_obstacle_env.py:61-71, sector_cr_env.py:53-66,
plan_waypoint_env.py:50-56.  Gymnasium's
spaces.Dict sorts its keys, and SB3's MultiInputPolicy flattens in that order, so the
flat fp32 row of libbsg is laid out in sorted-key order.
"""
from __future__ import annotations

import numpy as np

from . import _native as nat


def merge_sizes(k):
    return {"airspeed": 1, "cos(drift)": 1, "cos(track)": k, "distances": k,
            "faf_reached": 1, "sin(drift)": 1, "sin(track)": k, "vx_r": k, "vy_r": k,
            "waypoint_dist": 1, "x_r": k, "y_r": k}


def vertical_sizes(ni):
    return {"altitude": 1, "altitude_difference": ni, "cos_difference_pos": ni,
            "intruder_distance": ni, "runway_distance": 1, "sin_difference_pos": ni,
            "target_altitude": 1, "vz": 1, "x_difference_speed": ni,
            "y_difference_speed": ni, "z_difference_speed": ni}


def horizontal_sizes(ni):
    return {"cos_difference_pos": ni, "cos_drift": 1, "intruder_distance": ni,
            "sin_difference_pos": ni, "sin_drift": 1, "waypoint_distance": 1,
            "x_difference_speed": ni, "y_difference_speed": ni}


def static_sizes(nobst=10):
    return {"cos_difference_restricted_area_pos": nobst, "destination_waypoint_cos_drift": 1,
            "destination_waypoint_distance": 1, "destination_waypoint_sin_drift": 1,
            "restricted_area_distance": nobst, "restricted_area_radius": nobst,
            "sin_difference_restricted_area_pos": nobst}


def sector_sizes(k=4):
    return {"airspeed": 1, "cos(drift)": 1, "cos(track)": k, "distances": k, "sin(drift)": 1,
            "sin(track)": k, "vx_r": k, "vy_r": k, "x_r": k, "y_r": k}


def plan_sizes(nw=5):
    return {"cos_difference": nw, "sin_difference": nw, "waypoint_distance": nw,
            "waypoint_reached": nw}


def descent_sizes():
    return {"altitude": 1, "runway_distance": 1, "target_altitude": 1, "vz": 1}


# reference Box bounds (low, high) per key
_BOUNDS = {"cos(drift)": (-1, 1), "sin(drift)": (-1, 1), "faf_reached": (0, 1)}
_KIND_BOUNDS = {nat.ENV_SECTOR_CR: {"airspeed": (-1, 1)},
                nat.ENV_STATIC_OBSTACLE: {"restricted_area_radius": (0, 1)},
                nat.ENV_PLAN_WAYPOINT: {"waypoint_reached": (0, 1)}}


WIND_KEYS = ("wind_u", "wind_v")     # bluesky_gym/wrappers/wind.py:21-22

# insertion order of the observation dict each reference _get_obs builds (merge_env.py:222-
# 235, vertical_cr_env.py:162-178, descent_env.py:110-116, horizontal_cr_env.py:205-214);
# the dicts handed to users keep it (wrappers such as NoisyObservationWrapper draw their
# noise in this order), the flat rows use the sorted order
REF_ORDER = {
    nat.ENV_MERGE: ("cos(drift)", "sin(drift)", "airspeed", "waypoint_dist", "faf_reached",
                    "x_r", "y_r", "vx_r", "vy_r", "cos(track)", "sin(track)", "distances"),
    nat.ENV_VERTICAL_CR: ("altitude", "vz", "target_altitude", "runway_distance",
                          "intruder_distance", "cos_difference_pos", "sin_difference_pos",
                          "altitude_difference", "x_difference_speed", "y_difference_speed",
                          "z_difference_speed"),
    nat.ENV_DESCENT: ("altitude", "vz", "target_altitude", "runway_distance"),
    nat.ENV_HORIZONTAL_CR: ("intruder_distance", "cos_difference_pos", "sin_difference_pos",
                            "x_difference_speed", "y_difference_speed", "waypoint_distance",
                            "cos_drift", "sin_drift"),
    nat.ENV_STATIC_OBSTACLE: ("destination_waypoint_distance", "destination_waypoint_cos_drift",
                              "destination_waypoint_sin_drift", "restricted_area_radius",
                              "restricted_area_distance", "cos_difference_restricted_area_pos",
                              "sin_difference_restricted_area_pos"),
    nat.ENV_SECTOR_CR: ("cos(drift)", "sin(drift)", "airspeed", "x_r", "y_r", "vx_r", "vy_r",
                        "cos(track)", "sin(track)", "distances"),
    nat.ENV_PLAN_WAYPOINT: ("waypoint_distance", "cos_difference", "sin_difference",
                            "waypoint_reached"),
}


class ObsLayout:
    def __init__(self, kind, num_ac, num_ac_state, wind=False):
        if kind == nat.ENV_MERGE:
            sizes = merge_sizes(num_ac_state)
        elif kind == nat.ENV_VERTICAL_CR:
            sizes = vertical_sizes(num_ac - 1)
        elif kind == nat.ENV_HORIZONTAL_CR:
            sizes = horizontal_sizes(num_ac - 1)
        elif kind == nat.ENV_STATIC_OBSTACLE:
            sizes = static_sizes()
        elif kind == nat.ENV_SECTOR_CR:
            sizes = sector_sizes(num_ac_state)
        elif kind == nat.ENV_PLAN_WAYPOINT:
            sizes = plan_sizes()
        else:
            sizes = descent_sizes()
        if wind:
            sizes.update({k: 1 for k in WIND_KEYS})
        self.keys = tuple(sorted(sizes))
        self.ref_order = REF_ORDER[kind] + (WIND_KEYS if wind else ())
        self.bounds = {**_BOUNDS, **_KIND_BOUNDS.get(kind, {})}
        self.sizes = {k: sizes[k] for k in self.keys}
        off = 0
        self.slices = {}
        for k in self.keys:
            self.slices[k] = slice(off, off + self.sizes[k])
            off += self.sizes[k]
        self.dim = off

    def split(self, flat) -> dict:
        """[..., dim] -> {key: [..., size]} (float64 numpy, like the reference obs, in the
        reference's key insertion order)."""
        flat = np.asarray(flat, np.float64)
        return {k: flat[..., self.slices[k]] for k in self.ref_order}

    def observation_space(self, spaces):
        return spaces.Dict({k: spaces.Box(*self.bounds.get(k, (-np.inf, np.inf)), shape=(n,),
                                          dtype=np.float64)
                            for k, n in self.sizes.items()})
