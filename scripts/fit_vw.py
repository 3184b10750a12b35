#!/usr/bin/env python3
"""Coefficients of the executor's erfc-free v/w (csrc/rate_dev.h ``vw_pair``).

    python scripts/fit_vw.py            # prints the fp32 coefficients + the error table

v(t) = pdf(t) / cdf(t) is written through h(a) = 1 / R(a) - a, R the Mills ratio,
a = |t| (rate_dev.h has the two branches).  h is approximated as

    h(a) = r * P(s) / Q(s),   r = 1 / (a + 4),   s = a r  in [0, 1)

with deg P = 5, deg Q = 4: bounded on [0, inf) and decaying as 1/a, so no input
overflows it.  The fit is a linearised least-squares of the relative error,
reweighted by 1/Q (Sanathanan-Koerner iteration), against fp64 values of h (scipy
erfcx below a = 5, the Mills continued fraction above).  The table compares the
fp32 evaluation of the whole v/w against fp64 per range of t.
"""
import numpy as np
from scipy.special import erfcx

K = 4.0


def h_ref(a):
    a = np.asarray(a, dtype=np.float64)
    out = 1.0 / (np.sqrt(np.pi / 2) * erfcx(a / np.sqrt(2))) - a
    big = a > 5
    ab = a[big]
    f = ab.copy()
    for k in range(200, 1, -1):  # 1/R(a) - a = 1 / (a + 2 / (a + 3 / (a + ...)))
        f = ab + k / f
    out[big] = 1.0 / f
    return out


def fit(n=5, m=4, iters=40):
    s = np.concatenate([np.linspace(0, 1, 20001)[:-1], 1 - np.logspace(-9, -2, 2000)])
    a = K * s / (1 - s)
    y = h_ref(a) * (a + K)  # G(s) = h (a + K); G(1) = 1
    s, y = np.append(s, 1.0), np.append(y, 1.0)
    Q = np.ones_like(s)
    for _ in range(iters):
        A = np.vstack([s ** i for i in range(n + 1)] + [-y * s ** i for i in range(1, m + 1)]).T
        W = (1 / (np.abs(y) * np.abs(Q)))[:, None]
        sol, *_ = np.linalg.lstsq(A * W, y * W[:, 0], rcond=None)
        p, q = sol[:n + 1], np.concatenate([[1.0], sol[n + 1:]])
        Q = np.polyval(q[::-1], s)
    return p, q


def vw(t, p, q, dt):
    t = t.astype(dt)
    a = np.abs(t)
    r = dt(1) / (a + dt(K))
    s = a * r
    P, Qv = np.zeros_like(a), np.zeros_like(a)
    for c in p[::-1]:
        P = P * s + dt(c)
    for c in q[::-1]:
        Qv = Qv * s + dt(c)
    h = r * P * (dt(1) / Qv)
    phi = np.exp(-a * a * dt(0.5)) * dt(0.3989422804014327)
    D = a + h
    vp = phi * D * (dt(1) / (D - phi))
    neg = t <= 0
    v = np.where(neg, D, vp)
    return v, v * np.where(neg, h, vp + a)


def main():
    p, q = fit()
    print("P (s^0 .. s^5):", ", ".join("%.9ef" % np.float32(c) for c in p))
    print("Q (s^0 .. s^4):", ", ".join("%.9ef" % np.float32(c) for c in q))
    t = np.concatenate([np.linspace(-60, 15, 750001), -np.logspace(1, 6, 1000)])
    v32, w32 = vw(t, p, q, np.float32)
    a = np.abs(t)
    h = h_ref(a)
    D = a + h
    phi = np.exp(-a * a / 2) / np.sqrt(2 * np.pi)
    vp = phi * D / (D - phi)
    V = np.where(t <= 0, D, vp)
    W = V * np.where(t <= 0, h, vp + a)
    for lo, hi in ((-1e7, -5), (-5, 0), (0, 2), (2, 4), (4, 6), (6, 15)):
        m = (t >= lo) & (t < hi) & (V > 1e-30)
        print("t in [%g, %g): max rel err v %.2e  w %.2e" % (
            lo, hi, np.max(np.abs(v32[m] / V[m] - 1)), np.max(np.abs(w32[m] / W[m] - 1))))


if __name__ == "__main__":
    main()
