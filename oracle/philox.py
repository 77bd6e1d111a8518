"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- Philox4x32-10 counter RNG in NumPy.

Bit-identical restatement of the device RNG in
``bluesky-gym-hallucination_amd/csrc/bsg_device.h`` (``philox4x32_10``), used only so
that tests can reproduce the spawn parameters a device-side reset draws.  Algorithm:
Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11), 10 rounds,
multipliers 0xD2511F53 / 0xCD9E8D57, Weyl keys 0x9E3779B9 / 0xBB67AE85.

Counter layout used by every spawn draw: (env_id, episode, draw, tag).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

TAG_MERGE = 0x4D455247      # 'MERG'
TAG_VERT = 0x56455254       # 'VERT'
TAG_DESC = 0x44455343       # 'DESC'
TAG_HORZ = 0x484F525A       # 'HORZ'
TAG_PLAN = 0x504C414E       # 'PLAN'


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10.  c* broadcastable uint32 arrays, seed python int (64-bit).
    Returns 4 uint32 arrays."""
    c0 = np.asarray(c0, np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, np.uint32).astype(np.uint64)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for r in range(10):
            p0 = M0 * c0
            p1 = M1 * c2
            hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
            hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
            c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
            if r < 9:
                k0 = (k0 + np.uint64(W0)) & MASK32
                k1 = (k1 + np.uint64(W1)) & MASK32
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def u01_53(lo, hi):
    """Two uint32 -> double in [0, 1) with 53 random bits."""
    x = (np.asarray(hi, np.uint64) << np.uint64(32)) | np.asarray(lo, np.uint64)
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def randint_u32(x, lo, hi):
    """Integer in [lo, hi) from one uint32 by multiply-shift (exact integer math)."""
    lo = np.asarray(lo, np.int64)
    span = np.asarray(hi, np.int64) - lo
    return lo + ((np.asarray(x, np.uint64).astype(np.int64) * span) >> 32)
