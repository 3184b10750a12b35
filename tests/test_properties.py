"""Property-based tests (hypothesis) of the rating math and the batched engine."""
import math

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from analyzer_amd.models.trueskill import TrueSkill, v_w_win_closed
from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream

ENV = TrueSkill(mu=1500.0, sigma=1000.0, beta=1000.0, tau=10.0, draw_probability=0.0)
player = st.tuples(st.floats(-2000, 6000), st.floats(20, 1500))
team = st.lists(player, min_size=1, max_size=5)
SETTINGS = dict(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@settings(**SETTINGS)
@given(team, team)
def test_winner_gains_loser_loses_sigma_shrinks(a, b):
    na, nb = ENV.rate_two_teams(a, b, 0, 1)
    for (m0, s0), (m1, s1) in zip(a, na):
        assert m1 >= m0 - 1e-9 and s1 <= math.sqrt(s0 * s0 + 100.0) + 1e-9
    for (m0, s0), (m1, s1) in zip(b, nb):
        assert m1 <= m0 + 1e-9 and s1 <= math.sqrt(s0 * s0 + 100.0) + 1e-9


@settings(**SETTINGS)
@given(team, team)
def test_swapping_teams_mirrors_the_update(a, b):
    na, nb = ENV.rate_two_teams(a, b, 0, 1)
    mb, ma = ENV.rate_two_teams(b, a, 1, 0)
    for x, y in zip(na + nb, ma + mb):
        assert x[0] == pytest.approx(y[0], rel=1e-12, abs=1e-9)
        assert x[1] == pytest.approx(y[1], rel=1e-12)


@settings(**SETTINGS)
@given(team, team)
def test_quality_in_unit_interval_and_symmetric(a, b):
    q = ENV.quality_two_teams(a, b)
    assert 0.0 <= q <= 1.0
    assert q == pytest.approx(ENV.quality_two_teams(b, a), rel=1e-12)


@settings(**SETTINGS)
@given(st.floats(-60, 60))
def test_v_w_bounds(t):
    v, w = v_w_win_closed(t)
    # fp64: pdf(t) underflows past t ~ 37, where the exact update is < 1e-300 anyway
    assert v >= 0 and 0 <= w < 1
    if t < 30:
        assert v > 0 and w > 0
    assert w == pytest.approx(v * (v + t), rel=1e-9, abs=1e-300)


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(1, 5), st.integers(0, 2**31 - 1), st.floats(0, 0.3), st.floats(0, 0.3))
def test_host_engine_fp32_tracks_fp64(K, seed, p_tie, p_uneven):
    P = 30
    roster = make_roster(RosterSpec(num_players=P, seed=seed % 997))
    rec = make_stream(StreamSpec(team_size=K, seed=seed, p_tie=p_tie, p_uneven=p_uneven), 120, P, K=K)
    a, b = roster.clone(), roster.clone()
    ra = R.BatchRater(host_fp64=True).rate(a, rec, K)
    rb = R.BatchRater(host_fp64=False).rate(b, rec, K)
    assert torch.equal(ra.status, rb.status)
    np.testing.assert_allclose(rb.s_mu.numpy(), ra.s_mu.numpy(), rtol=2e-4, atol=0.05, equal_nan=True)
