"""Host side of the wind field: the table the device interpolates.

Mirrors ``bluesky.traffic.windfield.Windfield.addpointvne`` as driven by
``bluesky_gym/wrappers/wind.py:28`` (``bs.traf.wind.addpointvne(lat, lon, vnorth, veast,
alt)``): P points whose wind is constant in altitude (``alt=None``; ``vnorth``/``veast``
given as [P] or [1, P]) or given as profiles over ``alt`` ([len(alt), P]), which are
sampled onto the fixed altitude axis 0..45000 ft every 100 ft (np.interp, clamped at the
ends).  The lookup (``getdata``) runs on the device: bsg_kernels.hip ``wind_at``.
"""
from __future__ import annotations

import numpy as np

FT = 0.3048
ALTSTEP = 100.0 * FT
NALT = 451
ALTAXIS = np.arange(NALT, dtype=np.float64) * ALTSTEP


class WindTable:
    def __init__(self, lat, lon, vnorth, veast, alt=None):
        lat = np.atleast_1d(np.asarray(lat, np.float64)).ravel()
        lon = np.atleast_1d(np.asarray(lon, np.float64)).ravel()
        if lat.size != lon.size or lat.size == 0:
            raise ValueError("wind field: lat and lon must have the same, non-zero length")
        P = lat.size
        vn = np.asarray(vnorth, np.float64)
        ve = np.asarray(veast, np.float64)
        if alt is None:
            if vn.size != P or ve.size != P:
                raise ValueError(f"wind field: expected {P} wind values per component")
            vn, ve = vn.reshape(1, P), ve.reshape(1, P)
        else:
            wa = np.atleast_1d(np.asarray(alt, np.float64))
            vn, ve = vn.reshape(len(wa), P), ve.reshape(len(wa), P)
            vn = np.stack([np.interp(ALTAXIS, wa, vn[:, p]) for p in range(P)], 1)
            ve = np.stack([np.interp(ALTAXIS, wa, ve[:, p]) for p in range(P)], 1)
        self.lat, self.lon = lat, lon
        self.vnorth = np.ascontiguousarray(vn)
        self.veast = np.ascontiguousarray(ve)

    @property
    def num_points(self):
        return self.lat.size

    @property
    def num_levels(self):
        return self.vnorth.shape[0]
