"""Fit the polynomial of the fast ReLU covariance map (csrc/relu_poly.h).

The reference's ReLU map (kernels.py:146-152) is, with t = v1·v2 + tiny and
rho = clamp(c/sqrt(t), -1, 1),

    out = (sqrt(t - c²) + (π - acos rho)·c) / 2π .

Writing a = |rho| and x = (1 - a)/2 (so acos a = 2·asin(√x)) it is exactly

    out = max(c, 0)/2 + sqrt(t) · x·√x · P(x),
    P(x) = [ sqrt(1 - x) - (1 - 2x)·asin(√x)/√x ] / (π·x),         x ∈ [0, 1/2]

P is analytic on [0, 1/2] (its nearest singularity is x = 1), so one polynomial
covers every rho with no branch: Chebyshev convergence rate ρ_B = 3 + 2√2 ≈ 5.83 per
degree.  This script evaluates P in 50-digit decimal arithmetic (Taylor series of both
terms), interpolates at Chebyshev nodes of u = 4x - 1 ∈ [-1, 1], converts to monomials
in x itself (the kernels then need no u; Horner in x on [0, 1/2] is as accurate as in
u, because the singularity at x = 1 lies outside the disc |x| <= 1/2), rounds to
double/float and reports the max relative error of the rounded polynomial evaluated by
Horner in that precision.
"""
from decimal import Decimal, getcontext
from fractions import Fraction
import math

import numpy as np

getcontext().prec = 60
PI = Decimal("3.14159265358979323846264338327950288419716939937510582097494459")


def taylor_F_over_x(nterms=200):
    """Exact rational Taylor coefficients of F(x)/x, F(x) = sqrt(1-x) - (1-2x)·asin(√x)/√x."""
    # sqrt(1-x) = Σ binom(1/2, n) (-x)^n
    sq = []
    b = Fraction(1)
    for n in range(nterms + 2):
        sq.append(b * (-1) ** n)
        b = b * (Fraction(1, 2) - n) / (n + 1)
    # asin(√x)/√x = Σ C(2n,n)/(4^n (2n+1)) x^n
    asn = [Fraction(math.comb(2 * n, n), 4 ** n * (2 * n + 1)) for n in range(nterms + 2)]
    # (1-2x)·asn
    prod = [asn[n] - (2 * asn[n - 1] if n >= 1 else 0) for n in range(nterms + 2)]
    F = [sq[n] - prod[n] for n in range(nterms + 2)]
    assert F[0] == 0
    return F[1:nterms + 1]


COEF = taylor_F_over_x()


def P_dec(x: Decimal) -> Decimal:
    s = Decimal(0)
    p = Decimal(1)
    for c in COEF:
        s += Decimal(c.numerator) / Decimal(c.denominator) * p
        p *= x
    return s / PI


def fit(deg, xmax=0.5):
    """Chebyshev interpolation of P on x in [0, xmax] (u = 2x/xmax - 1 in [-1, 1]), high
    precision; returns monomials in u."""
    n = deg + 1
    X = Decimal(xmax)
    nodes = [Decimal(math.cos(math.pi * (k + 0.5) / n)) for k in range(n)]
    vals = [P_dec((u + 1) * X / 2) for u in nodes]
    cheb = []
    for j in range(n):
        s = Decimal(0)
        for k in range(n):
            s += vals[k] * Decimal(math.cos(math.pi * j * (k + 0.5) / n))
        cheb.append(s * 2 / n)
    cheb[0] /= 2
    # Chebyshev -> monomial in u (exact recurrence in Decimal)
    T = [[Decimal(1)], [Decimal(0), Decimal(1)]]
    for j in range(2, n):
        a = [Decimal(0)] + [2 * c for c in T[j - 1]]
        b = T[j - 2] + [Decimal(0)] * (len(a) - len(T[j - 2]))
        T.append([a[i] - b[i] for i in range(len(a))])
    mono = [Decimal(0)] * n
    for j in range(n):
        for i, c in enumerate(T[j]):
            mono[i] += cheb[j] * c
    return mono


def to_x(mono, xmax=0.5):
    """Monomials in u = 2x/xmax - 1 -> monomials in x (exact, in Decimal)."""
    out = [Decimal(0)] * len(mono)
    s = 2 / Decimal(xmax)
    for k, c in enumerate(mono):
        for j in range(k + 1):
            out[j] += c * math.comb(k, j) * s ** j * Decimal(-1) ** (k - j)
    return out


def horner(coefs, u, dt):
    r = dt(coefs[-1])
    for c in reversed(coefs[:-1]):
        r = r * u + dt(c)
    return r


def check(monox, dt, npts=20001, xmax=0.5):
    """Max relative error of the rounded x-monomials, Horner in dt over x in [0, xmax]."""
    cf = [dt(float(c)) for c in monox]
    worst = 0.0
    for k in range(npts):
        xd = dt(xmax * k / (npts - 1))
        ref = P_dec(Decimal(float(xd)))
        got = horner(cf, xd, dt)
        err = abs((Decimal(float(got)) - ref) / ref)
        worst = max(worst, float(err))
    return worst, cf


# range-adaptive ReLU (CGP_RELU_ADAPT): lower degrees on sub-intervals [0, xmax] with the
# same 1.6e-14 bound, taken by a wave whose every pixel has x <= xmax (relu_q_n)
ADAPT = ((0.125, 7), (0.25, 9), (0.375, 11))
# CGP_RELU_TOL=1: the same intervals at a 1e-12 bound (6 / 8 / 9, and 11 on [0, 1/2]:
# 2.2e-13 / 1.3e-13 / 9.2e-13 / 7.6e-13), 3-5 decades inside the end-to-end parity bounds
#  and 4 inside the reference's own acos noise near |rho| = 1
ADAPT_TOL = ((0.125, 6), (0.25, 8), (0.375, 9))
DEG_TOL = 11
# ... and for the float polynomial (its bound: the degree-6 fit's 7.9e-8)
ADAPT_F = ((0.125, 3), (0.375, 5))


def write_header(path, deg_d=13, deg_f=6, alt_d=(10, 11, 12)):
    """relu_poly.h: the double polynomial at deg_d (default) and, selectable with
    -DCGP_RELU_DEG_D=<n> for A/B builds, at each degree of alt_d; the float one at deg_f;
    the sub-interval polynomials of ADAPT."""
    mf = to_x(fit(deg_f))
    ef, cf = check(mf, np.float32, npts=4001)
    dbl = {}
    for d in sorted({deg_d, *alt_d}):
        dbl[d] = check(to_x(fit(d)), np.float64, npts=4001)
    sub = [(xm, d, check(to_x(fit(d, xm), xm), np.float64, npts=4001, xmax=xm))
           for xm, d in ADAPT]
    sub_tol = [(xm, d, check(to_x(fit(d, xm), xm), np.float64, npts=4001, xmax=xm))
               for xm, d in ADAPT_TOL]
    sub_f = [(xm, d, check(to_x(fit(d, xm), xm), np.float32, npts=4001, xmax=xm))
             for xm, d in ADAPT_F]
    lines = [
        "// relu_poly.h - generated by tools/fit_relu_poly.py --write (do not edit by hand).",
        "// P(x), x = (1 - |rho|)/2 in [0, 1/2], monomials in x; the fast ReLU covariance map is",
        "//   out = max(c, 0)/2 + sqrt(t) * x * sqrt(x) * P(x)",
        f"// double, on [0, 1/2] (CGP_RELU_DEG_D selects "
        + ", ".join(f"{d}: {dbl[d][0]:.2e}" for d in sorted(dbl)) + " max rel err);",
        f"// float: degree {deg_f}, max rel err {ef:.2e}",
        "#pragma once",
        "// CGP_RELU_TOL=1 (default): the 1e-12 tables (degree " + str(DEG_TOL)
        + " on [0, 1/2], adaptive " + " / ".join(str(d) for _, d in ADAPT_TOL)
        + "); CGP_RELU_TOL=0: the 1.6e-14 tables (degree " + str(deg_d) + ", adaptive "
        + " / ".join(str(d) for _, d in ADAPT) + ")",
        "#ifndef CGP_RELU_TOL",
        "#define CGP_RELU_TOL 1",
        "#endif",
        "#ifndef CGP_RELU_DEG_D",
        "#if CGP_RELU_TOL",
        f"#define CGP_RELU_DEG_D {DEG_TOL}",
        "#else",
        f"#define CGP_RELU_DEG_D {deg_d}",
        "#endif",
        "#endif",
    ]
    for k, d in enumerate(sorted(dbl)):
        lines += [f"#{'if' if k == 0 else 'elif'} CGP_RELU_DEG_D == {d}",
                  f"constexpr int kReluPolyDegD = {d};",
                  f"constexpr double kReluPolyD[{d + 1}] = {{"]
        lines += [f"    {float(c)!r}," for c in dbl[d][1]]
        lines += ["};"]
    lines += ["#else", "#error \"CGP_RELU_DEG_D: no table for this degree\"", "#endif"]
    for tag, rows in (("#if CGP_RELU_TOL", sub_tol), ("#else", sub)):
        lines += [tag]
        for k, (xm, d, (err, cfs)) in enumerate(rows):
            lines += [f"// x in [0, {xm}]: degree {d}, max rel err {err:.2e}",
                      f"constexpr double kReluAdaptX{k} = {xm!r};",
                      f"constexpr int kReluAdaptDeg{k} = {d};",
                      f"constexpr double kReluAdaptP{k}[{d + 1}] = {{"]
            lines += [f"    {float(c)!r}," for c in cfs]
            lines += ["};"]
    lines += ["#endif"]
    for k, (xm, d, (err, cfs)) in enumerate(sub_f):
        lines += [f"// float, x in [0, {xm}]: degree {d}, max rel err {err:.2e}",
                  f"constexpr float kReluAdaptFX{k} = {xm!r}f;",
                  f"constexpr int kReluAdaptFDeg{k} = {d};",
                  f"constexpr float kReluAdaptFP{k}[{d + 1}] = {{"]
        lines += [f"    {float(c)!r}f," for c in cfs]
        lines += ["};"]
    lines += [f"constexpr int kReluPolyDegF = {deg_f};",
              f"constexpr float kReluPolyF[{deg_f + 1}] = {{"]
    lines += [f"    {float(c)!r}f," for c in cf]
    lines += ["};", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))
    print("\n".join(lines))


if __name__ == "__main__":
    import os
    import sys
    if "--write" in sys.argv:
        here = os.path.dirname(os.path.abspath(__file__))
        write_header(os.path.join(here, "..", "cnn-gp_amd", "csrc", "relu_poly.h"))
    else:
        for name, dt, degs in (("double", np.float64, range(10, 19)),
                               ("float", np.float32, range(4, 9))):
            for deg in degs:
                err, cf = check(to_x(fit(deg)), dt, npts=3001)
                print(name, deg, f"max rel err {err:.3e}")
