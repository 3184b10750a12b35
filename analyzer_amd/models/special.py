"""Special functions behind TrueSkill's truncated-Gaussian moment matching.

Two numeric backends, selected by name exactly like the upstream ``trueskill``
package's ``backend=`` argument (used at /root/reference/rater.py:30-37):

* ``"float"`` (also ``None``): IEEE fp64 with numerically stable forms.  The
  Mills ratio is evaluated with a scaled complementary error function and a
  continued fraction in the far tail, so ``v``/``w`` stay finite where the naive
  ``pdf/cdf`` form under-/overflows.
* ``"mpmath"``: arbitrary precision through :mod:`mpmath` (the reference sets
  ``mpmath.mp.dps = 50`` at /root/reference/rater.py:7-8).

Both backends expose the same ``Numerics`` interface so the factor graph in
:mod:`analyzer_amd.models.factor_graph` is written once.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Callable

SQRT2 = math.sqrt(2.0)
SQRT2PI = math.sqrt(2.0 * math.pi)
INV_SQRTPI = 1.0 / math.sqrt(math.pi)


# --------------------------------------------------------------------------- fp64
def erfcx(x: float) -> float:
    """Scaled complementary error function ``exp(x*x) * erfc(x)``.

    For ``x >= 4`` the Laplace continued fraction is used, which keeps full
    relative precision long after ``erfc`` itself underflows (x > 26).
    """
    if x < 4.0:
        if x < -26.0:
            return math.inf
        return math.exp(x * x) * math.erfc(x)
    # erfc(x) = exp(-x^2)/sqrt(pi) * 1/(x + (1/2)/(x + 1/(x + (3/2)/(x + ...))))
    frac = x
    for k in range(60, 0, -1):
        frac = x + (k * 0.5) / frac
    return INV_SQRTPI / frac


def pdf(x: float) -> float:
    return math.exp(-0.5 * x * x) / SQRT2PI


def cdf(x: float) -> float:
    return 0.5 * math.erfc(-x / SQRT2)


def _mills_tail(u: float) -> float:
    """``h(u) = 1/(u + 2/(u + 3/(u + ...)))`` so that ``pdf(u)/Q(u) = u + h(u)``.

    ``Q`` is the upper normal tail.  Used for the far lower tail of ``v_win``
    where ``v = -t + h(-t)`` and ``w = v * h`` avoid the cancellation in
    ``v * (v + t)``.
    """
    frac = u
    for k in range(80, 1, -1):
        frac = u + k / frac
    return 1.0 / frac


def make_erfcinv(erfc, sqrt, log, exp):
    """Inverse of ``erfc``: rational first guess + two Halley-type corrections.

    This is the classic Numerical-Recipes scheme (the same family the upstream
    ``trueskill`` package uses).  Keeping its *finite* refinement matters for
    parity: with ``draw_probability=0`` the draw margin is ``ppf(0.5)``, which
    this scheme leaves at ~-2e-31 rather than exactly 0 under 50-digit mpmath,
    and that residual is what lets the reference rate tied matches at all
    (SURVEY App. C.7).
    """
    def erfcinv(y):
        if y >= 2:
            return -100.0
        if y <= 0:
            return 100.0
        lower = y < 1
        if not lower:
            y = 2 - y
        t = sqrt(-2 * log(y / 2.0))
        x = -0.70711 * ((2.30753 + t * 0.27061) / (1.0 + t * (0.99229 + t * 0.04481)) - t)
        for _ in range(2):
            err = erfc(x) - y
            x += err / (1.12837916709551257 * exp(-(x ** 2)) - x * err)
        return x if lower else -x
    return erfcinv


_erfcinv_f = make_erfcinv(math.erfc, math.sqrt, math.log, math.exp)


def ppf(p: float) -> float:
    """Inverse standard normal CDF."""
    return -SQRT2 * _erfcinv_f(2 * p)


def v_win_f(diff: float, margin: float) -> float:
    x = diff - margin
    if x < -5.0:
        u = -x
        return u + _mills_tail(u)
    # pdf(x)/cdf(x) == sqrt(2/pi) / erfcx(-x/sqrt2)
    return math.sqrt(2.0 / math.pi) / erfcx(-x / SQRT2)


def w_win_f(diff: float, margin: float) -> float:
    x = diff - margin
    if x < -5.0:
        u = -x
        h = _mills_tail(u)
        w = (u + h) * h
    else:
        v = v_win_f(diff, margin)
        w = v * (v + x)
    if 0.0 < w < 1.0:
        return w
    raise FloatingPointError("w_win out of (0, 1): diff=%r margin=%r" % (diff, margin))


def v_draw_f(diff: float, margin: float) -> float:
    ad = abs(diff)
    a, b = margin - ad, -margin - ad
    denom = cdf(a) - cdf(b)
    v = (pdf(b) - pdf(a)) / denom if denom else a
    return -v if diff < 0 else v


def w_draw_f(diff: float, margin: float) -> float:
    ad = abs(diff)
    a, b = margin - ad, -margin - ad
    denom = cdf(a) - cdf(b)
    if not denom:
        raise FloatingPointError("w_draw: empty draw interval (draw margin %r)" % margin)
    v = v_draw_f(ad, margin)
    return v * v + (a * pdf(a) - b * pdf(b)) / denom


# --------------------------------------------------------------------------- backend
@dataclass(frozen=True)
class Numerics:
    """Numeric backend used by the Gaussian/factor-graph code."""

    name: str
    cdf: Callable[[Any], Any]
    pdf: Callable[[Any], Any]
    ppf: Callable[[Any], Any]
    v_win: Callable[[Any, Any], Any]
    w_win: Callable[[Any, Any], Any]
    v_draw: Callable[[Any, Any], Any]
    w_draw: Callable[[Any, Any], Any]
    sqrt: Callable[[Any], Any]
    exp: Callable[[Any], Any]
    num: Callable[[Any], Any]  # coerce a python number into the backend type
    inf: Any


FLOAT = Numerics("float", cdf, pdf, ppf, v_win_f, w_win_f, v_draw_f, w_draw_f,
                 math.sqrt, math.exp, float, math.inf)


def _mpmath_numerics() -> Numerics:
    import mpmath

    m_erfcinv = make_erfcinv(mpmath.erfc, mpmath.sqrt, mpmath.log, mpmath.exp)

    def m_ppf(p):
        return -mpmath.sqrt(2) * m_erfcinv(2 * mpmath.mpf(p))

    def m_v_win(diff, margin):
        x = diff - margin
        denom = mpmath.ncdf(x)
        return mpmath.npdf(x) / denom if denom else -x

    def m_w_win(diff, margin):
        x = diff - margin
        v = m_v_win(diff, margin)
        w = v * (v + x)
        if 0 < w < 1:
            return w
        raise FloatingPointError("w_win out of (0, 1)")

    def m_v_draw(diff, margin):
        ad = abs(diff)
        a, b = margin - ad, -margin - ad
        denom = mpmath.ncdf(a) - mpmath.ncdf(b)
        v = (mpmath.npdf(b) - mpmath.npdf(a)) / denom if denom else a
        return -v if diff < 0 else v

    def m_w_draw(diff, margin):
        ad = abs(diff)
        a, b = margin - ad, -margin - ad
        denom = mpmath.ncdf(a) - mpmath.ncdf(b)
        if not denom:
            raise FloatingPointError("w_draw: empty draw interval")
        v = m_v_draw(ad, margin)
        return v * v + (a * mpmath.npdf(a) - b * mpmath.npdf(b)) / denom

    return Numerics("mpmath", mpmath.ncdf, mpmath.npdf, m_ppf, m_v_win, m_w_win,
                    m_v_draw, m_w_draw, mpmath.sqrt, mpmath.exp, mpmath.mpf, mpmath.inf)


def get_numerics(backend: str | None) -> Numerics:
    if backend in (None, "float", "fp64"):
        return FLOAT
    if backend == "mpmath":
        return _mpmath_numerics()
    raise ValueError("unsupported numeric backend %r (use 'float' or 'mpmath')" % (backend,))
