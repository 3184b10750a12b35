"""Numerics contract: golden vectors, EP == closed form, edge cases."""
import math
import random

import pytest

from analyzer_amd.config import RaterConfig
from analyzer_amd.models import special
from analyzer_amd.models.match_rater import MatchRater
from analyzer_amd.models.tiers import seed_from_attributes, vst_points
from analyzer_amd.models.trueskill import TrueSkill
from analyzer_amd.runtime.objects import Match, Participant, Player, Roster

ENV = TrueSkill(mu=1500, sigma=1000, beta=1000.0, tau=10.0, draw_probability=0)


def _match(mode, team0, team1, winners=(True, False), afk=()):
    def parts(players, base):
        return [Participant(p, "x%d" % (base + i), went_afk=1 if (base + i) in afk else 0)
                for i, p in enumerate(players)]

    r0 = Roster(parts(team0, 0), winner=winners[0])
    r1 = Roster(parts(team1, len(team0)), winner=winners[1])
    return Match(mode, [r0, r1], api_id="m")


def tier15():
    return Player(skill_tier=15)


# ----------------------------------------------------------------------- tiers
def test_vst_points_table():
    assert set(vst_points) == set(range(-1, 30))
    assert 30 not in vst_points
    assert vst_points[-1] == vst_points[0] == 1
    assert vst_points[15] == pytest.approx(1479.5455, abs=1e-4)
    assert vst_points[29] == pytest.approx(3079.5455, abs=1e-4)
    vals = [vst_points[t] for t in range(0, 30)]
    assert vals == sorted(vals)


def test_seed_rules():
    assert seed_from_attributes(None, None, 15, 500) == pytest.approx((1979.5454545, 500))
    mu, sig = seed_from_attributes(1200, None, 0, 500)
    assert (mu, sig) == pytest.approx((1533.3333333, 333.3333333))
    for rr, rb in ((2500, None), (2500, 100), (100, 2500), (None, 2500), (0, 2500)):
        mu, sig = seed_from_attributes(rr, rb, 0, 500)
        assert mu - sig == 2500
    with pytest.raises(KeyError):
        seed_from_attributes(None, None, 30, 500)
    with pytest.raises(KeyError):
        seed_from_attributes(0, 0, None, 500)


# ------------------------------------------------------------ special functions
def test_v_w_far_tail_stable():
    for t in (-4.9, -5.1, -8.0, -20.0, -40.0):
        v = special.v_win_f(t, 0.0)
        w = special.w_win_f(t, 0.0)
        assert v > -t and 0 < w < 1
    # w continuity across the branch switch
    assert special.w_win_f(-5.0 + 1e-9, 0.0) == pytest.approx(special.w_win_f(-5.0 - 1e-9, 0.0), rel=1e-7)


def test_v_w_match_mpmath():
    mp = special.get_numerics("mpmath")
    import mpmath

    mpmath.mp.dps = 40
    for t in (-30.0, -6.0, -2.0, 0.0, 1.5, 6.0):
        assert special.v_win_f(t, 0.0) == pytest.approx(float(mp.v_win(mpmath.mpf(t), 0)), rel=1e-12)
        assert special.w_win_f(t, 0.0) == pytest.approx(float(mp.w_win(mpmath.mpf(t), 0)), rel=1e-10)


def test_ppf_roundtrip():
    for p in (0.01, 0.3, 0.5, 0.9, 0.999):
        assert special.cdf(special.ppf(p)) == pytest.approx(p, rel=1e-9, abs=1e-12)


# ------------------------------------------------------ EP oracle == closed form
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_closed_form_equals_factor_graph(seed):
    rnd = random.Random(seed)
    for _ in range(60):
        A = [(rnd.uniform(0, 4000), rnd.uniform(30, 1000)) for _ in range(rnd.choice([1, 2, 3, 5]))]
        B = [(rnd.uniform(0, 4000), rnd.uniform(30, 1000)) for _ in range(rnd.choice([1, 3, 5]))]
        ranks = rnd.choice([(0, 1), (1, 0)])
        ca, cb = ENV.rate_two_teams(A, B, *ranks)
        ea, eb = ENV.rate([[ENV.create_rating(*x) for x in A], [ENV.create_rating(*x) for x in B]],
                          list(ranks))
        for (m, s), r in zip(ca + cb, list(ea) + list(eb)):
            assert m == pytest.approx(r.mu, rel=1e-11, abs=1e-9)
            assert s == pytest.approx(r.sigma, rel=1e-11)
        q = ENV.quality([[ENV.create_rating(*x) for x in A], [ENV.create_rating(*x) for x in B]])
        assert ENV.quality_two_teams(A, B) == pytest.approx(q, rel=1e-12)


def test_tie_limit_matches_50_digit_factor_graph():
    import mpmath

    mpmath.mp.dps = 50
    env = TrueSkill(mu=1500, sigma=1000, beta=1000.0, tau=10.0, draw_probability=0,
                    backend="mpmath")
    A, B = [(2300.0, 300.0)] * 3, [(1700.0, 250.0)] * 2
    ca, cb = ENV.rate_two_teams(A, B, 1, 1)
    ea, eb = env.rate([[env.create_rating(*x) for x in A], [env.create_rating(*x) for x in B]],
                      [1, 1])
    for (m, s), r in zip(ca + cb, list(ea) + list(eb)):
        assert m == pytest.approx(float(r.mu), rel=1e-12)
        assert s == pytest.approx(float(r.sigma), rel=1e-12)
    # float backend behaves like upstream's float backend: the empty draw interval raises
    with pytest.raises(FloatingPointError):
        ENV.rate([[ENV.create_rating(*x) for x in A], [ENV.create_rating(*x) for x in B]], [1, 1])


def test_multi_team_ep_runs_and_orders():
    env = TrueSkill()  # trueskill defaults (draws allowed)
    r = [env.create_rating() for _ in range(4)]
    out = env.rate([(r[0],), (r[1],), (r[2],), (r[3],)], ranks=[0, 1, 2, 3])
    mus = [g[0].mu for g in out]
    assert mus == sorted(mus, reverse=True)
    a, b = env.rate_1vs1(env.create_rating(), env.create_rating(), drawn=True)
    assert a.mu == pytest.approx(b.mu, abs=1e-9)
    assert 0 < env.quality_1vs1(env.create_rating(), env.create_rating()) <= 1


# ------------------------------------------------------------- golden vectors
def _rater(backend="closed"):
    return MatchRater(RaterConfig(backend=backend))


@pytest.mark.parametrize("backend", ["closed", "ep"])
def test_golden_g1_new_players(backend):
    team0 = [tier15() for _ in range(3)]
    team1 = [tier15() for _ in range(3)]
    m = _match("ranked", team0, team1)
    _rater(backend).rate_match(m)
    assert m.trueskill_quality == pytest.approx(0.894427191, abs=1e-9)
    for p in m.rosters[0].participants:
        pl = p.player[0]
        assert pl.trueskill_mu == pytest.approx(2052.408237, abs=1e-5)
        assert pl.trueskill_sigma == pytest.approx(494.763595, abs=1e-5)
        assert pl.trueskill_ranked_mu == pytest.approx(2052.408237, abs=1e-5)
        assert p.trueskill_delta == 0
    for p in m.rosters[1].participants:
        assert p.player[0].trueskill_mu == pytest.approx(1906.682672, abs=1e-5)


def test_golden_g2_returning_players():
    mk = lambda: Player(trueskill_mu=2000.0, trueskill_sigma=100.0)  # noqa: E731
    m = _match("ranked", [mk() for _ in range(3)], [mk() for _ in range(3)])
    _rater().rate_match(m)
    assert m.trueskill_quality == pytest.approx(0.99503719021, abs=1e-10)
    w, l = m.rosters[0].participants[0], m.rosters[1].participants[0]
    assert w.player[0].trueskill_mu == pytest.approx(2003.273434, abs=1e-5)
    assert w.player[0].trueskill_sigma == pytest.approx(100.445431, abs=1e-5)
    assert w.trueskill_delta == pytest.approx(2.828003, abs=1e-5)
    assert l.trueskill_delta == pytest.approx(-3.718865, abs=1e-5)
    assert w.player[0].trueskill_ranked_mu == pytest.approx(2003.273434, abs=1e-5)


def test_golden_g3_upset_mixed_seeds():
    r0 = [Player(skill_tier=0, rank_points_ranked=1200), Player(skill_tier=0, rank_points_blitz=1300),
          Player(trueskill_mu=1400.0, trueskill_sigma=200.0, trueskill_ranked_mu=1350.0,
                 trueskill_ranked_sigma=150.0)]
    r1 = [Player(skill_tier=0, rank_points_ranked=2500), Player(skill_tier=29),
          Player(trueskill_mu=2600.0, trueskill_sigma=120.0, trueskill_ranked_mu=2700.0,
                 trueskill_ranked_sigma=90.0)]
    m = _match("ranked", r0, r1)
    _rater().rate_match(m)
    assert m.trueskill_quality == pytest.approx(0.192871830817, abs=1e-10)
    expect = [
        (1625.385186, 331.050170, 0, 1627.861480, 331.029261),
        (1725.385186, 331.050170, 0, 1727.861480, 331.029261),
        (1433.191641, 199.724259, 33.467382, 1369.209736, 150.108811),
        (2741.281481, 331.050170, 0, 2738.805186, 331.029261),
        (3372.532252, 491.856321, 0, 3366.963372, 491.785144),
        (2587.998035, 120.301760, -12.303725, 2693.030096, 90.504885),
    ]
    for p, (smu, ssig, d, rmu, rsig) in zip(m.participants, expect):
        pl = p.player[0]
        assert pl.trueskill_mu == pytest.approx(smu, abs=1e-5)
        assert pl.trueskill_sigma == pytest.approx(ssig, abs=1e-5)
        assert p.trueskill_delta == pytest.approx(d, abs=1e-5)
        assert pl.trueskill_ranked_mu == pytest.approx(rmu, abs=1e-5)
        assert pl.trueskill_ranked_sigma == pytest.approx(rsig, abs=1e-5)
        assert p.participant_items[0].trueskill_ranked_mu == pytest.approx(rmu, abs=1e-5)


# ------------------------------------------------------------------ edge cases
def test_unsupported_mode_writes_nothing():
    m = _match("private", [tier15()], [tier15()])
    _rater().rate_match(m)
    assert m.trueskill_quality is None
    assert all(p.player[0].trueskill_mu is None for p in m.participants)


def test_afk_and_invalid_rosters():
    m = _match("ranked", [tier15() for _ in range(3)], [tier15() for _ in range(3)], afk={4})
    _rater().rate_match(m)
    assert m.trueskill_quality == 0
    assert all(p.participant_items[0].any_afk for p in m.participants)
    assert all(p.player[0].trueskill_mu is None for p in m.participants)
    m = _match("ranked", [tier15()], [tier15()])
    m.rosters.append(Roster([], winner=False))
    _rater().rate_match(m)
    assert m.trueskill_quality == 0 and all(p.participant_items[0].any_afk for p in m.participants)


def test_error_classes():
    with pytest.raises(KeyError):
        _rater().rate_match(_match("ranked", [Player(skill_tier=30)], [tier15()]))
    m = _match("ranked", [tier15()], [])
    with pytest.raises(ValueError):
        _rater().rate_match(m)
    with pytest.raises(ValueError):
        _rater().rate_match(_match("ranked", [Player(trueskill_mu=1000.0, trueskill_sigma=0.0)],
                                   [tier15()]))


def test_tie_none_winner_and_uneven():
    a, b = Player(trueskill_mu=2300.0, trueskill_sigma=300.0), Player(trueskill_mu=1700.0, trueskill_sigma=300.0)
    m = _match("casual", [a], [b], winners=(False, False))
    _rater().rate_match(m)
    assert a.trueskill_mu < 2300 and b.trueskill_mu > 1700  # draw pulls them together
    a2, b2 = tier15(), tier15()
    m = _match("casual", [a2], [b2], winners=(None, True))  # None loses
    _rater().rate_match(m)
    assert b2.trueskill_mu > a2.trueskill_mu
    m = _match("ranked", [tier15()], [tier15()])
    _rater().rate_match(m)
    assert m.trueskill_quality == pytest.approx(0.894, abs=1e-3)
    m = _match("ranked", [tier15(), tier15()], [tier15(), tier15(), tier15()])
    _rater().rate_match(m)
    assert m.trueskill_quality == pytest.approx(0.654, abs=1e-3)


def test_aliased_player_in_match_follows_write_order():
    # the reference's fixtures repeat one participant object: later writes win and the
    # second occurrence's delta is taken against the first occurrence's write
    same = Player(trueskill_mu=2000.0, trueskill_sigma=100.0)
    other = [Player(trueskill_mu=2000.0, trueskill_sigma=100.0) for _ in range(3)]
    m = _match("ranked", [same, same, same], other)
    _rater().rate_match(m)
    d = [p.trueskill_delta for p in m.rosters[0].participants]
    assert d[0] == pytest.approx(2.828003, abs=1e-5)
    assert d[1] == pytest.approx(0.0, abs=1e-9) and d[2] == pytest.approx(0.0, abs=1e-9)
