"""Gaussian messages in natural parameters and the user-facing ``Rating``.

``Gaussian`` stores precision ``pi = 1/sigma^2`` and precision-adjusted mean
``tau = mu/sigma^2``: products and quotients of Gaussians (the only algebra
expectation propagation needs) are then additions/subtractions.  The number
type is whatever the active numeric backend hands in (python float or mpmath
``mpf``), so the same code runs the fp64 oracle and the 50-digit mode that
/root/reference/rater.py:6-8 selects.
"""
from __future__ import annotations

import math
from typing import Any


class Gaussian:
    __slots__ = ("pi", "tau")

    def __init__(self, mu: Any = None, sigma: Any = None, pi: Any = 0, tau: Any = 0):
        if mu is not None:
            if sigma is None:
                raise TypeError("sigma argument is needed")
            if sigma == 0:
                # same error class and message family as trueskill.Gaussian
                raise ValueError("sigma**2 should be greater than 0")
            pi = sigma ** -2
            tau = pi * mu
        self.pi = pi
        self.tau = tau

    @property
    def mu(self):
        return self.pi and self.tau / self.pi

    @property
    def sigma(self):
        return self.pi ** -0.5 if self.pi else math.inf

    def __mul__(self, other: "Gaussian") -> "Gaussian":
        return Gaussian(pi=self.pi + other.pi, tau=self.tau + other.tau)

    def __truediv__(self, other: "Gaussian") -> "Gaussian":
        return Gaussian(pi=self.pi - other.pi, tau=self.tau - other.tau)

    def __eq__(self, other):  # pragma: no cover - convenience
        return isinstance(other, Gaussian) and self.pi == other.pi and self.tau == other.tau

    def __hash__(self):  # pragma: no cover
        return hash((self.pi, self.tau))

    def __repr__(self) -> str:
        return "N(mu=%.6f, sigma=%.6f)" % (float(self.mu), float(self.sigma))


class Rating(Gaussian):
    """A player's skill belief N(mu, sigma^2)."""

    __slots__ = ()

    def __init__(self, mu: Any = None, sigma: Any = None):
        if isinstance(mu, tuple):
            mu, sigma = mu
        elif isinstance(mu, Gaussian):
            mu, sigma = mu.mu, mu.sigma
        super().__init__(mu, sigma)

    def __iter__(self):
        yield self.mu
        yield self.sigma

    def __float__(self) -> float:
        return float(self.mu)

    def __repr__(self) -> str:
        return "Rating(mu=%.3f, sigma=%.3f)" % (float(self.mu), float(self.sigma))
