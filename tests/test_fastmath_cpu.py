"""CPU checks of the kernel's fixed-exponent powers and constant atmospheres (no GPU).

bsg_fastmath.h replaces the device libm pow of the atmosphere / CAS-TAS chain
(oracle/bluesky_subset.py vatmos, vtas2cas, vcas2tas) by Chebyshev polynomials; the
device/host bit-identity and the ulp statistics against glibc are measured by
tools/probe/fastmath_probe.hip (profiles/r02/fastmath_probe.txt).  Here: the generated
coefficients approximate the powers they claim to (exact binary64 exponents), and the
two constant atmospheres hard-coded in bsg_device.h are the oracle's vatmos values.
"""
import os
import re

import numpy as np
import pytest

from oracle import bluesky_subset as bs

CSRC = os.path.join(os.path.dirname(__file__), "..", "bluesky-gym-hallucination_amd", "csrc")


def _coeffs():
    txt = open(os.path.join(CSRC, "bsg_fastmath_coeffs.h")).read()
    out = {}
    for name in ("T", "35", "27"):
        x0 = float(re.search(rf"kPow{name}_X0 = ([^;]+);", txt).group(1))
        lo, hi = (float(v) for v in re.search(rf"kPow{name}_LO = ([^,]+), kPow{name}_HI = ([^;]+);", txt).groups())
        body = re.search(rf"kPow{name}_C\[\d+\] = \{{[^\n]*\n(.*?)\}};", txt, re.S).group(1)
        cs = [float(v) for v in re.findall(r"(-?[\d.]+e?-?\d*),", body)]
        clo = [float(v) for v in re.search(rf"kPow{name}_CLO\[3\] = \{{([^}}]+)\}}", txt).group(1).split(",")]
        out[name] = (x0, lo, hi, cs, clo)
    return out


@pytest.mark.parametrize("name,expo", [("T", 4.256848030018761), ("35", 3.5), ("27", 2.0 / 7.0)])
def test_fastpow_coefficients_approximate_the_power(name, expo):
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 40
    x0, lo, hi, cs, clo = _coeffs()[name]
    cs = [mp.mpf(c) for c in cs]
    for k in range(3):
        cs[len(cs) - 3 + k] += mp.mpf(clo[k])
    worst = 0
    for x in np.linspace(lo, hi, 257):
        d = mp.mpf(float(x)) - mp.mpf(x0)
        p = mp.mpf(0)
        for c in cs:
            p = p * d + c
        ref = mp.mpf(float(x)) ** mp.mpf(expo)
        worst = max(worst, abs(p / ref - 1))
    assert worst < 1e-17, float(worst)


def test_constant_atmospheres_are_the_oracle_vatmos():
    txt = open(os.path.join(CSRC, "bsg_device.h")).read()
    for name, h in (("kAtmosHMAX", bs.HMAX), ("kAtmosSL", 0.0)):
        lits = re.search(rf"constexpr Atmos {name} = \{{([^}}]+)\}};", txt).group(1).split(",")
        got = [float.fromhex(v.strip()) for v in lits]
        want = [float(v) for v in bs.vatmos(np.float64(h))]
        assert got == want, (name, got, want)


def test_constant_atmosphere_divisors():
    """kAtmos*_K: the divisors PerfModel.limits' conversions use at the two constant
    atmospheres and their RN reciprocals (bsg_device.h AtmosK), as the host computes them."""
    txt = open(os.path.join(CSRC, "bsg_device.h")).read()
    for name, h in (("kAtmosHMAX_K", bs.HMAX), ("kAtmosSL_K", 0.0)):
        body = re.search(rf"constexpr AtmosK {name} = \{{(\w+),([^}}]+)\}};", txt, re.S)
        got = [float.fromhex(v.strip()) for v in body.group(2).split(",")]
        p, rho, T = (float(v) for v in bs.vatmos(np.float64(h)))
        p7 = 7.0 * p
        snd = float(np.sqrt(1.4 * 287.05287 * T))
        want = [p7, 1.0 / p7, 1.0 / p, p7 / rho, snd, 1.0 / snd]
        assert got == want, (name, got, want)


def test_constant_atmosphere_clamp_thresholds():
    """kLim*: PerfModel.limits' CAS clamp at the two constant atmospheres as TAS values --
    vcas2tas(vmin), vcas2tas(vmax), vcas2tas(vmax_gd) -- exactly as the oracle (NumPy)
    computes them (bsg_device.h LimK), and ordered as the clamp needs."""
    txt = open(os.path.join(CSRC, "bsg_device.h")).read()
    for name, h in (("kLimHMAX", bs.HMAX), ("kLimSL", 0.0)):
        lits = re.search(rf"constexpr LimK {name} = \{{([^}}]+)\}};", txt).group(1).split(",")
        got = [float.fromhex(v.strip()) for v in lits]
        want = [float(bs.vcas2tas(np.float64(c), np.float64(h)))
                for c in (bs.VMIN_CAS, bs.VMAX_CAS, bs.VMAX_GD)]
        assert got == want, (name, got, want)
        assert 0.0 < got[0] < got[1]
    # the round trip the threshold form replaces: NumPy's tas -> cas -> tas at the constant
    # atmospheres returns its argument within 1e-13 relative over the flown speed range
    for h in (bs.HMAX, 0.0):
        tas = np.linspace(60.0, 300.0, 2001)
        rt = bs.vcas2tas(bs.vtas2cas(tas, np.float64(h)), np.float64(h))
        assert np.max(np.abs(rt / tas - 1.0)) < 1e-13
