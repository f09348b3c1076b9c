"""Coefficients of the fp64 fast transcendentals in csrc/adrp_device.h (f64 namespace), fitted
here in extended precision (numpy longdouble, 64-bit mantissa) and checked against the
longdouble libm:

  atan(t) = t + t^3 P(t^2) on |t| <= tan(pi/8)      (after the octant / pi/4 reduction)
  exp(r)  = Taylor to r^13 on |r| <= ln2/2           (after k = rint(x log2 e))
  sin/cos = Taylor to x^13 / x^14 on |x| <= pi/8     (the exp-map half angle is clamped there)

Least squares on Chebyshev nodes (near-minimax).  Prints the C literals and the max errors of a
float64 Horner evaluation (each step rounded to double, as the FMA chain does at worst).
"""
import numpy as np

L = np.longdouble


def cheb_nodes(a, b, n):
    k = np.arange(n, dtype=L)
    return (a + b) / 2 + (b - a) / 2 * np.cos((2 * k + 1) * L(np.pi) / (2 * n))


def fit_atan(deg):
    """P(s) = (atan(t) - t) / t^3, s = t^2: least squares in the Chebyshev basis of the mapped
    variable u = 2 s / smax - 1 (well conditioned), residual refinement in longdouble, then the
    series is re-expanded in powers of s in longdouble"""
    tmax = L("0.41421356237309504880")
    smax = tmax * tmax
    s = cheb_nodes(L(0), smax, 4000)
    t = np.sqrt(s)
    f = (np.arctan(t) - t) / (t * s)
    u = 2 * s / smax - 1
    T = np.polynomial.chebyshev.chebvander(u.astype(np.float64), deg).astype(L)
    # Chebyshev recurrence in longdouble for the refinement residuals
    TL = np.empty((len(u), deg + 1), dtype=L)
    TL[:, 0] = 1
    TL[:, 1] = u
    for k in range(2, deg + 1):
        TL[:, k] = 2 * u * TL[:, k - 1] - TL[:, k - 2]
    a = np.zeros(deg + 1, dtype=L)
    for _ in range(4):
        r = f - TL @ a
        da, *_ = np.linalg.lstsq(T.astype(np.float64), r.astype(np.float64), rcond=None)
        a = a + da.astype(L)
    # sum a_k T_k(u), u = alpha s - 1  ->  power series in s (longdouble polynomial arithmetic)
    alpha = 2 / smax
    Pprev = np.zeros(deg + 1, dtype=L); Pprev[0] = 1                  # T0
    Pcur = np.zeros(deg + 1, dtype=L); Pcur[0] = -1; Pcur[1] = alpha    # T1
    c = a[0] * Pprev + a[1] * Pcur
    for k in range(2, deg + 1):
        nxt = np.zeros(deg + 1, dtype=L)
        nxt[1:] += 2 * alpha * Pcur[:-1]
        nxt -= 2 * Pcur
        nxt -= Pprev
        c = c + a[k] * nxt
        Pprev, Pcur = Pcur, nxt
    return c.astype(np.float64)


def horner(c, x):
    p = np.float64(c[-1])
    for k in range(len(c) - 2, -1, -1):
        p = np.float64(p * x + c[k])
    return p


def check_atan(c):
    t = np.linspace(-0.41421356237309504880, 0.41421356237309504880, 200001)
    s = t * t
    got = t + t * s * np.array([horner(c, x) for x in s[::50]]).repeat(1)[:0].sum() if False else None
    P = np.zeros_like(s)
    p = np.full_like(s, c[-1])
    for k in range(len(c) - 2, -1, -1):
        p = p * s + c[k]
    got = t + t * s * p
    ref = np.arctan(t.astype(L))
    err = np.abs(got.astype(L) - ref) / np.maximum(np.abs(ref), L(1e-300))
    return float(np.max(err[t != 0]))


def check_exp():
    r = np.linspace(-0.34657359027997264, 0.34657359027997264, 200001)
    c = [1.0 / float(np.prod(np.arange(1, k + 1, dtype=L))) for k in range(14)]
    p = np.full_like(r, c[-1])
    for k in range(len(c) - 2, -1, -1):
        p = p * r + c[k]
    ref = np.exp(r.astype(L))
    return float(np.max(np.abs(p.astype(L) - ref) / ref)), c


def check_sincos():
    x = np.linspace(-0.39269908169872414, 0.39269908169872414, 200001)
    x2 = x * x
    sc = [(-1) ** k / float(np.prod(np.arange(1, 2 * k + 2, dtype=L))) for k in range(7)]
    cc = [(-1) ** k / float(np.prod(np.arange(1, 2 * k + 1, dtype=L))) for k in range(8)]
    ps = np.full_like(x, sc[-1])
    for k in range(len(sc) - 2, -1, -1):
        ps = ps * x2 + sc[k]
    s = x * ps
    pc = np.full_like(x, cc[-1])
    for k in range(len(cc) - 2, -1, -1):
        pc = pc * x2 + cc[k]
    xs = x.astype(L)
    es = np.abs(s.astype(L) - np.sin(xs))[x != 0] / np.abs(np.sin(xs))[x != 0]
    ec = np.abs(pc.astype(L) - np.cos(xs)) / np.cos(xs)
    return float(es.max()), float(ec.max()), sc, cc


if __name__ == "__main__":
    for deg in (9, 10, 11, 12):
        c = fit_atan(deg)
        print(f"atan deg {deg}: max rel err {check_atan(c):.3e}")
    c = fit_atan(9)
    print("atan P coefficients (s^0 .. s^9):")
    print(", ".join(repr(float(v)) for v in c))
    e, ce = check_exp()
    print(f"exp Taylor r^13 max rel err {e:.3e}")
    es, ec, sc, cc = check_sincos()
    print(f"sin x^13 max rel err {es:.3e}, cos x^14 {ec:.3e}")
    print("sin:", ", ".join(repr(v) for v in sc))
    print("cos:", ", ".join(repr(v) for v in cc))
    print("exp:", ", ".join(repr(v) for v in ce))
