"""The executor's erfc-free v/w (csrc/rate_dev.h ``vw_pair``), evaluated on the host in
fp32 with the coefficients parsed from the header, against the 50-digit mpmath values
of v = pdf(t)/cdf(t), w = v (v + t) that the reference computes
(/root/reference/rater.py:8, trueskill's v_win / w_win).  Guards the header's constants
(scripts/fit_vw.py derives them)."""
import math
import os
import re

import numpy as np
import pytest

HDR = os.path.join(os.path.dirname(__file__), "..", "analyzer_amd", "csrc", "rate_dev.h")


def _coefficients():
    src = open(HDR).read()
    body = src[src.index("void vw_pair"):src.index("const f2 h = r * P * rcp2(Q);")]
    lit = r"(-?\d+\.\d+e[+-]\d+)f"
    p = [float(re.search(r"f2 P = f2\{" + lit, body).group(1))]
    p += [float(x) for x in re.findall(r"P = P \* s \+ " + lit, body)]
    q = [float(re.search(r"f2 Q = f2\{" + lit, body).group(1))]
    q += [float(x) for x in re.findall(r"Q = Q \* s \+ " + lit, body)] + [1.0]
    k = float(re.search(r"constexpr float kK = ([\d.]+)f", body).group(1))
    return p, q, k  # highest power first (Horner order)


def _vw32(t, p, q, k):
    f = np.float32
    t = np.asarray(t, dtype=f)
    a = np.abs(t)
    r = f(1) / (a + f(k))
    s = a * r
    P = np.full_like(a, f(p[0]))
    for c in p[1:]:
        P = P * s + f(c)
    Q = np.full_like(a, f(q[0]))
    for c in q[1:]:
        Q = Q * s + f(c)
    h = r * P * (f(1) / Q)
    phi = np.exp2(a * a * f(-0.72134752044448170)) * f(0.39894228040143268)
    D = a + h
    vp = phi * D * (f(1) / (D - phi))
    v = np.where(t <= 0, D, vp)
    w = v * np.where(t <= 0, h, vp + a)
    return v.astype(np.float64), w.astype(np.float64)


def test_header_coefficients_parse():
    p, q, k = _coefficients()
    assert len(p) == 6 and len(q) == 5 and k == 4.0
    assert abs(p[-1] / q[-1] / k - math.sqrt(2 / math.pi)) < 1e-6  # h(0) = v(0) = 2 phi(0)


@pytest.mark.parametrize("t", [-40.0, -12.0, -5.0, -2.5, -1.0, -0.25, 0.0, 0.3, 1.0, 2.0, 3.5])
def test_vw_matches_mpmath(t):
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 50
    T = mp.mpf(t)
    v_ref = mp.npdf(T) / mp.ncdf(T)
    w_ref = v_ref * (v_ref + T)
    v, w = _vw32([t], *_coefficients())
    assert abs(v[0] / float(v_ref) - 1) < 1.5e-6, (t, v[0], float(v_ref))
    assert abs(w[0] / float(w_ref) - 1) < 1.5e-6, (t, w[0], float(w_ref))


def test_vw_limits():
    p, q, k = _coefficients()
    v, w = _vw32([-1e6, 20.0, 60.0], p, q, k)
    assert abs(v[0] - 1e6) / 1e6 < 1e-6 and abs(w[0] - 1.0) < 1e-5  # big upset: v ~ -t, w -> 1
    assert v[1] == 0.0 and w[1] == 0.0 and v[2] == 0.0  # pdf underflow: the exact v = w = 0 limit
