"""The error bound k_stack_linfit decides LINEARFIT's clips with (sg_stack.hip, lfx_pixel_m).

The kernel takes the fit from exact integer sums and decides each `line_clipping` test
(src/stacking/stacking.c:1170-1183) only when it lies outside a bound on how far the reference's
rounded `gsl_fit_linear` recurrences (:1750-1784) can be from the exact fit.  This CPU test pins
that bound: on random and adversarial sorted stacks it runs GSL's double recurrences exactly as
the reference does (numpy float64 scalars, the same operation order), computes the exact slope,
intercept and mean absolute residual with rationals, and checks that every deviation stays within
the per-quantity bounds the kernel uses before the 4x safety factor on each test's margin (on these
stacks the largest observed error is 2.3e-3 of its bound: intercept; 4.3e-4 slope, 2.4e-4 sigma).
"""
from fractions import Fraction

import numpy as np
import pytest

U = 2.0 ** -53


def gsl_fit(y):
    """gsl_fit_linear(x = 0..n-1, y) as the reference calls it: (intercept, slope)."""
    n = len(y)
    f = np.float64
    m_x = m_y = m_dx2 = m_dxdy = f(0.0)
    for i in range(n):
        m_x += (f(i) - m_x) / (f(i) + f(1.0))
        m_y += (f(y[i]) - m_y) / (f(i) + f(1.0))
    for i in range(n):
        dx = f(i) - m_x
        dy = f(y[i]) - m_y
        m_dx2 += (dx * dx - m_dx2) / (f(i) + f(1.0))
        m_dxdy += (dx * dy - m_dxdy) / (f(i) + f(1.0))
    b = m_dxdy / m_dx2
    a = m_y - m_x * b
    return a, b


def ref_sigma(y, a, b):
    """the reference's sigma: sum of fabs(y - (slope * i + intercept)) / N, in order"""
    f = np.float64
    s = f(0.0)
    for i, v in enumerate(y):
        s += abs(f(v) - (b * f(i) + a))
    return s / f(len(y))


def exact_fit(y):
    n = len(y)
    sy = sum(int(v) for v in y)
    siy = sum(i * int(v) for i, v in enumerate(y))
    slope = Fraction(12 * siy - 6 * (n - 1) * sy, n * (n * n - 1))
    icpt = Fraction(sy, n) - Fraction(n - 1, 2) * slope
    sig = sum(abs(Fraction(int(v)) - (slope * i + icpt)) for i, v in enumerate(y)) / n
    return slope, icpt, sig


def bounds(n, Y, slope, b0):
    """the bounds of lfx_pixel_m before its 4x factor and closed-form rounding up"""
    as_ = abs(slope)
    dmx, dmy = 2.0 * n * n * U, 2.0 * n * U * Y
    dmdx2, dmdxdy = 6.0 * n ** 3 * U, 6.0 * n * n * U * Y
    mdx2 = (n * n - 1.0) / 12.0
    dS = (dmdxdy + as_ * dmdx2) / (mdx2 - dmdx2) + 4.0 * U * as_
    Rm = Y + n * as_ + abs(b0) + 1.0
    dB = dmy + as_ * dmx + 0.5 * n * dS + 8.0 * U * Rm
    dline = n * dS + dB + 32.0 * U * Rm
    dsig = dline + 2.0 * (n + 2.0) * U * Rm
    return dS, dB, dline, dsig


def stacks():
    rng = np.random.default_rng(7)
    out = []
    for n in (8, 16, 33, 100, 257, 512):
        for kind in ("noise", "outliers", "bright", "ramp", "steps", "wide"):
            if kind == "noise":
                y = rng.normal(1000, 30, n)
            elif kind == "outliers":
                y = rng.normal(2000, 50, n)
                k = max(1, n // 20)
                y[rng.choice(n, k, replace=False)] = rng.integers(20000, 65536, k)
            elif kind == "bright":
                y = rng.normal(64000, 900, n)
            elif kind == "ramp":
                y = 100 + 37 * np.arange(n) + rng.integers(0, 3, n)
            elif kind == "steps":
                y = rng.choice([0, 1200, 1201, 65535], n, p=[0.05, 0.45, 0.45, 0.05])
            else:
                y = rng.integers(0, 65536, n)
            out.append(np.sort(np.clip(np.rint(y), 0, 65535).astype(np.int64)))
    return out


@pytest.mark.parametrize("idx", range(36))
def test_reference_recurrences_within_bound(idx):
    y = stacks()[idx]
    n, Y = len(y), float(y.max())
    a_ref, b_ref = gsl_fit(y)                     # intercept, slope
    s_ref = ref_sigma(y, a_ref, b_ref)
    slope, icpt, sig = exact_fit(y)
    dS, dB, dline, dsig = bounds(n, Y, float(slope), float(icpt))
    assert abs(Fraction(float(b_ref)) - slope) <= Fraction(dS), (n, float(b_ref), float(slope), dS)
    assert abs(Fraction(float(a_ref)) - icpt) <= Fraction(dB), (n, float(a_ref), float(icpt), dB)
    # each line value the clip test forms, a * i + b with the reference's doubles
    f = np.float64
    worst = max(abs(Fraction(float(b_ref * f(i) + a_ref)) - (slope * i + icpt)) for i in range(n))
    assert worst <= Fraction(dline), (n, float(worst), dline)
    assert abs(Fraction(float(s_ref)) - sig) <= Fraction(dsig), (n, float(s_ref), float(sig), dsig)


def test_bound_is_not_vacuous():
    """the bounds stay far below the clip scale (a sigma of ~30 ADU), so the fast path decides
    almost every test: at N = 512, Y = 65535 every bound is under 1e-5"""
    dS, dB, dline, dsig = bounds(512, 65535.0, 120.0, 2000.0)
    assert 4 * dline < 1e-5 and 4 * dsig < 1e-4


def test_closed_form_covers_bound():
    """lfx_pixel_m rounds the bounds up to closed forms; they must not fall below the derivation"""
    for n in (8, 9, 16, 100, 512, 1024):
        for Y in (1.0, 300.0, 65535.0):
            for s in (0.0, 0.01, 3.0, 1.75 * Y / n):
                for b0 in (0.0, Y, -Y):
                    dS, dB, dline, dsig = bounds(n, Y, s, b0)
                    as_ = abs(s)
                    kS = 98.0 * U * (Y + n * as_ + as_)
                    Rm = Y + n * as_ + abs(b0) + 1.0
                    kB = 2.0 * U * n * (Y + n * as_) + 0.5 * n * kS + 8.0 * U * Rm
                    assert kS >= dS and kB >= dB, (n, Y, s, kS, dS, kB, dB)
