"""CPU check of the closed-form ReLU covariance map used by the HIP kernels
(csrc/relu_poly.h): out = max(c,0)/2 + sqrt(t)·x·sqrt(x)·P(x), x = (1-|rho|)/2.

The kernel evaluates exactly this expression (with a Newton-refined hardware rsqrt);
here it is emulated in numpy float64 with the generated coefficients and compared with
(a) the reference's op-by-op formula (kernels.py:146-152, via the oracle) and (b) a
50-digit evaluation of the exact map."""
import os
import re
import sys
from decimal import Decimal, getcontext

import numpy as np

from oracle import nngp_oracle as O

from conftest import PKG

HDR = os.path.join(PKG, "csrc", "relu_poly.h")


def default_degree():
    """The double degree on [0, 1/2] the default build compiles: CGP_RELU_TOL (default 1)
    picks the first CGP_RELU_DEG_D default (the 1e-12 tables), else the second."""
    txt = open(HDR).read()
    tol = int(re.search(r"#define CGP_RELU_TOL (\d+)", txt).group(1))
    degs = [int(d) for d in re.findall(r"#define CGP_RELU_DEG_D (\d+)", txt)]
    return degs[0] if tol else degs[1]


# max relative error of the default double polynomial (relu_poly.h: degree 11, 7.6e-13;
# degree 13 with CGP_RELU_TOL=0, 1.6e-14)
BOUND_D = {11: 7.7e-13, 13: 1.6e-14}


def coeffs(kind, deg=None):
    """The coefficient table the default build compiles (the double one is selected by
    CGP_RELU_DEG_D among several degrees; ``deg`` picks another)."""
    txt = open(HDR).read()
    n = r"\d+"
    if kind == "D":
        n = str((deg or default_degree()) + 1)
    body = re.search(r"kReluPoly%s\[%s\] = \{(.*?)\};" % (kind, n), txt, re.S).group(1)
    return [float(v.strip().rstrip("f")) for v in body.split(",") if v.strip()]


def adapt_tables(tol):
    """(xmax, coefficients) of the range-adaptive fits in the CGP_RELU_TOL = tol branch"""
    txt = open(HDR).read()
    a = txt.index("#if CGP_RELU_TOL\n// x in")
    b = txt.index("#else", a)
    c = txt.index("#endif", b)
    blk = txt[a:b] if tol else txt[b:c]
    xs = [float(v) for v in re.findall(r"kReluAdaptX\d = ([0-9.]+);", blk)]
    ps = [[float(v) for v in body.split(",") if v.strip()]
          for body in re.findall(r"kReluAdaptP\d\[\d+\] = \{(.*?)\};", blk, re.S)]
    return list(zip(xs, ps))


def closed_form(c, v1, v2, cf, dt=np.float64):
    c, v1, v2 = (np.asarray(a, dtype=dt) for a in (c, v1, v2))
    t = v1 * v2 + dt(O.F32_TINY)
    y = dt(1) / np.sqrt(t)
    st = t * y
    a = np.minimum(np.abs(c * y), dt(1))
    x = dt(0.5) - dt(0.5) * a
    sx = np.sqrt(x)
    p = np.full_like(x, dt(cf[-1]))
    for k in reversed(cf[:-1]):
        p = p * x + dt(k)
    return (st * x) * sx * p + dt(0.5) * np.maximum(c, dt(0))


def reference_formula(c, v1, v2):
    kp = O.make_kp(False, True, np.asarray(c)[:, None, None], np.asarray(v1)[:, None, None],
                   np.asarray(v2)[:, None, None])
    return O.relu(kp)["xy"].reshape(-1)


def exact_dec(c, v1, v2):
    getcontext().prec = 50
    c, v1, v2 = Decimal(float(c)), Decimal(float(v1)), Decimal(float(v2))
    t = v1 * v2 + Decimal(O.F32_TINY)
    rho = c / t.sqrt()
    rho = max(min(rho, Decimal(1)), Decimal(-1))
    # acos via atan of the half-angle: acos r = 2 atan(sqrt((1-r)/(1+r)))
    import math
    th = Decimal(2) * Decimal(math.atan(float(((1 - rho) / (1 + rho)).sqrt()))) \
        if rho > -1 else Decimal(math.pi)
    s = (t - c * c).sqrt() if t > c * c else Decimal(0)
    pi = Decimal("3.14159265358979323846264338327950288419716939937510")
    return float((s + (pi - th) * c) / (2 * pi))


def test_closed_form_matches_reference_formula():
    rng = np.random.default_rng(0)
    n = 200000
    v1 = rng.lognormal(0, 2, n)
    v2 = rng.lognormal(0, 2, n)
    rho = rng.uniform(-1, 1, n)
    # stress the ends of [-1, 1] too
    rho[:2000] = 1 - 10 ** rng.uniform(-16, -1, 2000)
    rho[2000:4000] = -1 + 10 ** rng.uniform(-16, -1, 2000)
    c = rho * np.sqrt(v1 * v2)
    got = closed_form(c, v1, v2, coeffs("D"))
    ref = reference_formula(c, v1, v2)
    scale = np.sqrt(v1 * v2)       # the map's natural magnitude
    err = np.abs(got - ref) / scale
    # away from |rho| = 1 both are accurate to a few ulps of sqrt(t)
    mid = np.abs(rho) < 0.999
    # (the polynomial's own bound plus a few ulps: degree 13 gave 1e-14)
    assert err[mid].max() < max(1e-14, BOUND_D[default_degree()]), err[mid].max()
    # near |rho| = 1 the reference's acos(rho) carries ~sqrt(eps) noise
    assert err.max() < 3e-8, err.max()


def test_closed_form_known_answers():
    cf = coeffs("D")
    s6 = np.sqrt(6.0)
    got = closed_form([0.0, s6, -s6, 0.0], [2.0, 2.0, 2.0, 0.0], [3.0, 3.0, 3.0, 0.0], cf)
    # rho = 0 is the end x = 1/2 of the fit, where the polynomial is furthest off
    # (relu_poly.h: 1.5e-14 relative at degree 13, 7.6e-13 at the default 11)
    bound = max(2e-14, BOUND_D[default_degree()])
    assert abs(got[0] - s6 / (2 * np.pi)) < bound * s6 / (2 * np.pi)
    assert abs(got[1] - s6 / 2) < 1e-15          # exact here (the reference: 4e-9 off)
    assert abs(got[2]) < 1e-15
    assert abs(got[3] - 1.7255613506e-20) / 1.7255613506e-20 < 1e-9


def test_closed_form_against_50_digit_map():
    cf = coeffs("D")
    rng = np.random.default_rng(1)
    for _ in range(300):
        v1, v2 = rng.lognormal(0, 1, 2)
        rho = rng.uniform(-0.999, 0.999)
        c = rho * np.sqrt(v1 * v2)
        got = closed_form([c], [v1], [v2], cf)[0]
        ref = exact_dec(c, v1, v2)
        assert abs(got - ref) <= max(4e-15, BOUND_D[default_degree()]) * np.sqrt(v1 * v2), \
            (rho, got, ref)


def test_float_closed_form():
    cf = coeffs("F")
    rng = np.random.default_rng(2)
    v1 = rng.lognormal(0, 1, 50000).astype(np.float32)
    v2 = rng.lognormal(0, 1, 50000).astype(np.float32)
    rho = rng.uniform(-1, 1, 50000)
    c = (rho * np.sqrt(v1.astype(np.float64) * v2)).astype(np.float32)
    got = closed_form(c, v1, v2, cf, np.float32).astype(np.float64)
    ref = reference_formula(c.astype(np.float64), v1.astype(np.float64), v2.astype(np.float64))
    err = np.abs(got - ref) / np.sqrt(v1.astype(np.float64) * v2)
    assert err.max() < 2e-6, err.max()


def test_adaptive_tables_hold_their_bounds():
    """The range-adaptive sub-interval fits (relu_q_n's votes): the default CGP_RELU_TOL=1
    tables (degrees 6 / 8 / 9 on [0, 1/8] / [0, 1/4] / [0, 3/8]) within 1e-12 of the exact
    P, the CGP_RELU_TOL=0 ones (7 / 9 / 11) within 1e-14"""
    getcontext().prec = 50
    sys.path.insert(0, os.path.join(os.path.dirname(PKG), "tools"))
    from fit_relu_poly import P_dec
    for tol, bound, degs in ((1, 1e-12, [6, 8, 9]), (0, 1e-14, [7, 9, 11])):
        tabs = adapt_tables(tol)
        assert [len(p) - 1 for _, p in tabs] == degs
        assert [x for x, _ in tabs] == [0.125, 0.25, 0.375]
        for xmax, p in tabs:
            x = np.linspace(0.0, xmax, 129)
            got = np.full_like(x, p[-1])
            for k in reversed(p[:-1]):
                got = got * x + k
            ref = np.array([float(P_dec(Decimal(float(v)))) for v in x])
            assert np.max(np.abs(got - ref) / ref) < bound, (tol, xmax)
