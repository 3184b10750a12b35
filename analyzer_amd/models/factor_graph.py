"""General n-team TrueSkill expectation propagation (the CPU oracle).

This is the semantics of the ``trueskill==0.4.4`` engine that the reference
calls at /root/reference/rater.py:141,144,161 (E3-E7 in SURVEY.md §2.2),
rebuilt from the published algorithm (Herbrich et al., "TrueSkill: A Bayesian
Skill Rating System"; Minka's EP):

  skill_i  --Prior(+tau^2)-->  rating var
  rating   --Likelihood(+beta^2)-->  performance var
  perf     --Sum(weights)-->  team performance
  team_k, team_k+1  --Sum(+1,-1)-->  difference  --Truncate(v/w)-->

The schedule: one downward sweep, an EP loop over the difference chain (one
pass for two teams, forward+backward passes otherwise, at most 10 iterations,
stop when the largest message change <= ``min_delta``), then the upward sweep.

This module is the *reference oracle*, not the production path: production
rating of two-team matches runs the closed form on MI355X (csrc/rate_kernels.hip),
which SURVEY App. A.3 shows is identical to this EP for two teams.
"""
from __future__ import annotations

from typing import Any, List, Sequence

from .gaussian import Gaussian
from .special import Numerics


class Variable(Gaussian):
    """A marginal plus the last message each neighbouring factor sent."""

    __slots__ = ("messages",)

    def __init__(self):
        super().__init__()
        self.messages: dict = {}

    def _set(self, value: Gaussian, num: Numerics):
        pi_delta = abs(self.pi - value.pi)
        if pi_delta == num.inf:
            delta = 0
        else:
            delta = max(abs(self.tau - value.tau), num.sqrt(pi_delta))
        self.pi, self.tau = value.pi, value.tau
        return delta

    def update_message(self, factor, pi, tau, num: Numerics):
        old = self.messages[factor]
        msg = Gaussian(pi=pi, tau=tau)
        self.messages[factor] = msg
        return self._set(self / old * msg, num)

    def update_value(self, factor, pi, tau, num: Numerics):
        old = self.messages[factor]
        value = Gaussian(pi=pi, tau=tau)
        self.messages[factor] = value * old / self
        return self._set(value, num)


class _Factor:
    def __init__(self, variables: Sequence[Variable]):
        self.vars = list(variables)
        for v in self.vars:
            v.messages[self] = Gaussian()


class PriorFactor(_Factor):
    def __init__(self, var, value, dynamic, num):
        super().__init__([var])
        self.value, self.dynamic, self.num = value, dynamic, num

    def down(self):
        sigma = self.num.sqrt(self.value.sigma ** 2 + self.dynamic ** 2)
        g = Gaussian(self.value.mu, sigma)
        return self.vars[0].update_value(self, g.pi, g.tau, self.num)


class LikelihoodFactor(_Factor):
    def __init__(self, mean_var, value_var, variance, num):
        super().__init__([mean_var, value_var])
        self.mean, self.value, self.variance, self.num = mean_var, value_var, variance, num

    def _send(self, src: Variable, dst: Variable):
        msg = src / src.messages[self]
        a = 1 / (1 + self.variance * msg.pi)
        return dst.update_message(self, a * msg.pi, a * msg.tau, self.num)

    def down(self):
        return self._send(self.mean, self.value)

    def up(self):
        return self._send(self.value, self.mean)


class SumFactor(_Factor):
    """``sum = sum_k coeffs[k] * terms[k]``."""

    def __init__(self, sum_var, term_vars, coeffs, num):
        super().__init__([sum_var] + list(term_vars))
        self.sum, self.terms, self.coeffs, self.num = sum_var, list(term_vars), list(coeffs), num

    def _update(self, target, vals, coeffs):
        pi_inv = 0
        mu = 0
        for val, coeff in zip(vals, coeffs):
            div = val / val.messages[self]
            mu += coeff * div.mu
            if pi_inv == self.num.inf:
                continue
            if div.pi == 0:
                pi_inv = self.num.inf
            else:
                pi_inv += coeff ** 2 / div.pi
        pi = 1 / pi_inv
        return target.update_message(self, pi, pi * mu, self.num)

    def down(self):
        return self._update(self.sum, self.terms, self.coeffs)

    def up(self, index: int):
        coeff = self.coeffs[index]
        coeffs = []
        for k, c in enumerate(self.coeffs):
            if coeff == 0:
                coeffs.append(0)
            elif k == index:
                coeffs.append(1 / coeff)
            else:
                coeffs.append(-c / coeff)
        vals = list(self.terms)
        vals[index] = self.sum
        return self._update(self.terms[index], vals, coeffs)


class TruncateFactor(_Factor):
    def __init__(self, var, v_func, w_func, draw_margin, num):
        super().__init__([var])
        self.v_func, self.w_func, self.margin, self.num = v_func, w_func, draw_margin, num

    def up(self):
        var = self.vars[0]
        div = var / var.messages[self]
        sqrt_pi = self.num.sqrt(div.pi)
        t, eps = div.tau / sqrt_pi, self.margin * sqrt_pi
        v = self.v_func(t, eps)
        w = self.w_func(t, eps)
        denom = 1 - w
        return var.update_value(self, div.pi / denom, (div.tau + sqrt_pi * v) / denom, self.num)


def run_ep(sorted_groups: List[Sequence[Gaussian]], sorted_ranks: Sequence[Any],
           sorted_weights: List[Sequence[Any]], *, beta, tau, draw_probability,
           num: Numerics, min_delta=0.0001, max_iter: int = 10):
    """Run the TrueSkill factor graph; returns posterior (mu, sigma) per group.

    Inputs are already sorted by rank (best first), as in ``TrueSkill.rate``.
    """
    flat = [r for g in sorted_groups for r in g]
    flat_w = [w for ws in sorted_weights for w in ws]
    n_teams = len(sorted_groups)
    size = len(flat)
    rating_vars = [Variable() for _ in range(size)]
    perf_vars = [Variable() for _ in range(size)]
    team_vars = [Variable() for _ in range(n_teams)]
    diff_vars = [Variable() for _ in range(n_teams - 1)]
    sizes = [len(g) for g in sorted_groups]
    starts = [sum(sizes[:k]) for k in range(n_teams)]

    priors = [PriorFactor(v, r, tau, num) for v, r in zip(rating_vars, flat)]
    likes = [LikelihoodFactor(rv, pv, beta ** 2, num) for rv, pv in zip(rating_vars, perf_vars)]
    team_sums = [
        SumFactor(team_vars[k], perf_vars[starts[k]:starts[k] + sizes[k]],
                  flat_w[starts[k]:starts[k] + sizes[k]], num)
        for k in range(n_teams)
    ]
    diff_sums = [SumFactor(diff_vars[k], team_vars[k:k + 2], [1, -1], num)
                 for k in range(n_teams - 1)]
    truncs = []
    for k in range(n_teams - 1):
        pair = sizes[k] + sizes[k + 1]
        margin = num.ppf((draw_probability + 1) / 2.0) * num.sqrt(num.num(pair)) * beta
        if sorted_ranks[k] == sorted_ranks[k + 1]:
            vf, wf = num.v_draw, num.w_draw
        else:
            vf, wf = num.v_win, num.w_win
        truncs.append(TruncateFactor(diff_vars[k], vf, wf, margin, num))

    for f in priors:
        f.down()
    for f in likes:
        f.down()
    for f in team_sums:
        f.down()
    nd = len(diff_sums)
    for _ in range(max_iter):
        if nd == 1:
            diff_sums[0].down()
            delta = truncs[0].up()
        else:
            delta = 0
            for k in range(nd - 1):
                diff_sums[k].down()
                delta = max(delta, truncs[k].up())
                diff_sums[k].up(1)
            for k in range(nd - 1, 0, -1):
                diff_sums[k].down()
                delta = max(delta, truncs[k].up())
                diff_sums[k].up(0)
        if delta <= min_delta:
            break
    diff_sums[0].up(0)
    diff_sums[nd - 1].up(1)
    for f in team_sums:
        for k in range(len(f.terms)):
            f.up(k)
    for f in likes:
        f.up()

    out = []
    for k in range(n_teams):
        out.append([(rv.mu, rv.sigma) for rv in rating_vars[starts[k]:starts[k] + sizes[k]]])
    return out
