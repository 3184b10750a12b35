"""TrueSkill environment: the rating model the reference runs.

``TrueSkill`` mirrors the constructor and methods the reference uses on its
``env`` object (/root/reference/rater.py:30-37, 121, 132, 141, 144, 161):
``create_rating``, ``rate(groups, ranks)`` and ``quality(groups)``, plus the
usual 1-vs-1 helpers.  Two code paths produce the same numbers:

* ``rate`` / ``quality``: general n-team expectation propagation over the
  factor graph in :mod:`.factor_graph` (fp64 or mpmath backend);
* ``rate_two_teams`` / ``quality_two_teams``: the closed form for two teams
  (SURVEY App. A.3/A.4), which is what the MI355X kernels implement.  The EP
  result for two teams equals it (the EP loop converges after one truncation
  update), so the closed form is exact, not an approximation.
"""
from __future__ import annotations

import math
from itertools import chain
from typing import Any, Iterable, List, Optional, Sequence, Tuple

from .factor_graph import run_ep
from .gaussian import Gaussian, Rating
from .special import SQRT2, erfcx, get_numerics, _mills_tail

MU = 25.0
SIGMA = MU / 3
BETA = SIGMA / 2
TAU = SIGMA / 100
DRAW_PROBABILITY = 0.10
DELTA = 0.0001


def _is_mapping(x) -> bool:
    return hasattr(x, "keys") and hasattr(x, "values")


def v_w_win_closed(t: float) -> Tuple[float, float]:
    """Stable ``v = pdf(t)/cdf(t)`` and ``w = v (v + t)`` in fp64 (zero draw margin)."""
    if t < -5.0:
        u = -t
        h = _mills_tail(u)
        return u + h, (u + h) * h
    v = math.sqrt(2.0 / math.pi) / erfcx(-t / SQRT2)
    return v, v * (v + t)


class TrueSkill:
    """Rating environment (mu, sigma, beta, tau, draw_probability, backend)."""

    def __init__(self, mu: float = MU, sigma: float = SIGMA, beta: float = BETA,
                 tau: float = TAU, draw_probability: float = DRAW_PROBABILITY,
                 backend: Optional[str] = None):
        self.mu = mu
        self.sigma = sigma
        self.beta = beta
        self.tau = tau
        self.draw_probability = draw_probability
        self.backend = backend
        self.num = get_numerics(backend)

    # ------------------------------------------------------------------ basics
    def create_rating(self, mu: Any = None, sigma: Any = None) -> Rating:
        if mu is None:
            mu = self.mu
        if sigma is None:
            sigma = self.sigma
        return Rating(mu, sigma)

    def expose(self, rating: Gaussian) -> float:
        """Conservative skill estimate (mu - k*sigma with k = mu0/sigma0)."""
        k = self.mu / self.sigma
        return rating.mu - k * rating.sigma

    def cdf(self, x):
        return self.num.cdf(x)

    def pdf(self, x):
        return self.num.pdf(x)

    def ppf(self, x):
        return self.num.ppf(x)

    def __repr__(self):
        return ("TrueSkill(mu=%.3f, sigma=%.3f, beta=%.3f, tau=%.3f, draw_probability=%.3f, "
                "backend=%r)" % (self.mu, self.sigma, self.beta, self.tau,
                                 self.draw_probability, self.backend))

    # -------------------------------------------------------------- validation
    def validate_rating_groups(self, rating_groups):
        keys = None
        groups = list(rating_groups)
        if len(groups) < 2:
            raise ValueError("Need multiple rating groups")
        if not all(len(g) if not _is_mapping(g) else len(g.keys()) for g in groups):
            raise ValueError("Each group must contain multiple ratings")
        if _is_mapping(groups[0]):
            keys = [list(g.keys()) for g in groups]
            groups = [[g[k] for k in ks] for g, ks in zip(groups, keys)]
        else:
            groups = [list(g) for g in groups]
        return groups, keys

    def _weights(self, weights, groups, keys):
        if weights is None:
            return [[1] * len(g) for g in groups]
        if _is_mapping(weights):
            out = [[1] * len(g) for g in groups]
            for (gi, key), w in weights.items():
                idx = keys[gi].index(key) if keys is not None else key
                out[gi][idx] = w
            return out
        return [list(w) for w in weights]

    # -------------------------------------------------------------- rate (EP)
    def rate(self, rating_groups, ranks: Optional[Sequence[Any]] = None,
             weights=None, min_delta: float = DELTA):
        groups, keys = self.validate_rating_groups(rating_groups)
        ws = self._weights(weights, groups, keys)
        n = len(groups)
        if ranks is None:
            ranks = list(range(n))
        elif len(ranks) != n:
            raise ValueError("Wrong ranks")
        order = sorted(range(n), key=lambda k: ranks[k])  # stable
        s_groups = [groups[k] for k in order]
        s_ranks = [ranks[k] for k in order]
        s_weights = [[max(min_delta, w) for w in ws[k]] for k in order]
        num = self.num
        res = run_ep(s_groups, s_ranks, s_weights, beta=num.num(self.beta),
                     tau=num.num(self.tau), draw_probability=num.num(self.draw_probability),
                     num=num, min_delta=min_delta)
        out: List[Any] = [None] * n
        for pos, k in enumerate(order):
            out[k] = tuple(Rating(float(mu), float(sigma)) for mu, sigma in res[pos])
        if keys is not None:
            return [dict(zip(ks, g)) for ks, g in zip(keys, out)]
        return out

    # ---------------------------------------------------------- quality (EP)
    def quality(self, rating_groups, weights=None) -> float:
        groups, keys = self.validate_rating_groups(rating_groups)
        ws = self._weights(weights, groups, keys)
        flat = list(chain.from_iterable(groups))
        flat_w = list(chain.from_iterable(ws))
        n = len(groups)
        # A: players x (teams-1) comparison matrix; quality = N(0 | A^T mu, beta^2 A^T A + A^T S A)
        import numpy as np

        sizes = [len(g) for g in groups]
        A = np.zeros((len(flat), n - 1))
        start = 0
        for k in range(n - 1):
            for i in range(sizes[k]):
                A[start + i, k] = flat_w[start + i]
            nxt = start + sizes[k]
            for i in range(sizes[k + 1]):
                A[nxt + i, k] = -flat_w[nxt + i]
            start = nxt
        mu = np.array([float(r.mu) for r in flat])
        var = np.diag([float(r.sigma) ** 2 for r in flat])
        ata = (self.beta ** 2) * A.T @ A
        atsa = A.T @ var @ A
        middle = ata + atsa
        start_v = mu @ A
        e_arg = -0.5 * start_v @ np.linalg.inv(middle) @ start_v
        s_arg = np.linalg.det(ata) / np.linalg.det(middle)
        return math.exp(e_arg) * math.sqrt(s_arg)

    # --------------------------------------------------------- 1 vs 1 helpers
    def rate_1vs1(self, rating1, rating2, drawn: bool = False, min_delta: float = DELTA):
        ranks = [0, 0 if drawn else 1]
        a, b = self.rate([(rating1,), (rating2,)], ranks, min_delta=min_delta)
        return a[0], b[0]

    def quality_1vs1(self, rating1, rating2) -> float:
        return self.quality([(rating1,), (rating2,)])

    # ------------------------------------------------------ two-team closed form
    def rate_two_teams(self, team_a: Sequence[Tuple[float, float]],
                       team_b: Sequence[Tuple[float, float]], rank_a: int, rank_b: int):
        """Closed-form two-team update with ``draw_probability == 0``.

        ``team_*`` are sequences of (mu, sigma).  Equal ranks take the exact
        epsilon->0 draw limit (what the reference computes at 50 digits).
        Returns two lists of (mu, sigma).
        """
        if not team_a or not team_b:
            raise ValueError("Each group must contain multiple ratings")
        if self.draw_probability != 0:
            ra, rb = self.rate([[Rating(*r) for r in team_a], [Rating(*r) for r in team_b]],
                               [rank_a, rank_b])
            return [tuple(map(float, r)) for r in ra], [tuple(map(float, r)) for r in rb]
        b2 = float(self.beta) ** 2
        t2 = float(self.tau) ** 2
        for _, s in chain(team_a, team_b):
            if s == 0:
                raise ValueError("sigma**2 should be greater than 0")
        s2a = [s * s + t2 for _, s in team_a]
        s2b = [s * s + t2 for _, s in team_b]
        n = len(team_a) + len(team_b)
        c2 = n * b2 + sum(s2a) + sum(s2b)
        c = math.sqrt(c2)
        d = sum(m for m, _ in team_a) - sum(m for m, _ in team_b)
        if rank_a == rank_b:
            # draw limit: v = -t, w = 1
            ka = [-s * d / c2 for s in s2a]
            kb = [s * d / c2 for s in s2b]
            wa = wb = 1.0
            new_a = [(m + k, math.sqrt(s * (1 - s / c2 * wa)))
                     for (m, _), k, s in zip(team_a, ka, s2a)]
            new_b = [(m + k, math.sqrt(s * (1 - s / c2 * wb)))
                     for (m, _), k, s in zip(team_b, kb, s2b)]
            return new_a, new_b
        sign = 1.0 if rank_a < rank_b else -1.0
        t = sign * d / c
        v, w = v_w_win_closed(t)
        if not 0.0 < w < 1.0:
            raise FloatingPointError("w_win out of (0, 1)")
        new_a = [(m + sign * s / c * v, math.sqrt(s * (1 - s / c2 * w)))
                 for (m, _), s in zip(team_a, s2a)]
        new_b = [(m - sign * s / c * v, math.sqrt(s * (1 - s / c2 * w)))
                 for (m, _), s in zip(team_b, s2b)]
        return new_a, new_b

    def quality_two_teams(self, team_a: Sequence[Tuple[float, float]],
                          team_b: Sequence[Tuple[float, float]]) -> float:
        """Closed-form two-team match quality (sigma without tau)."""
        if not team_a or not team_b:
            raise ValueError("Each group must contain multiple ratings")
        n = len(team_a) + len(team_b)
        b2n = n * float(self.beta) ** 2
        denom = b2n + sum(s * s for _, s in chain(team_a, team_b))
        d = sum(m for m, _ in team_a) - sum(m for m, _ in team_b)
        return math.sqrt(b2n / denom) * math.exp(-d * d / (2.0 * denom))


def global_env() -> TrueSkill:  # pragma: no cover - convenience like trueskill.global_env
    return _GLOBAL


_GLOBAL = TrueSkill()
