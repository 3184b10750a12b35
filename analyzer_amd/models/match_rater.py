"""Object-level match rating: the reference's ``rate_match`` contract.

Operates on any objects exposing the ORM attribute names the reference touches
(SQLAlchemy rows from :mod:`analyzer_amd.runtime.store`, or plain Python
fixtures like the reference's tests): ``match.game_mode/rosters/participants/
trueskill_quality``, ``roster.winner/participants``, ``participant.went_afk/
player[0]/participant_items[0]/trueskill_{mu,sigma,delta}`` and the
``player.trueskill[_<mode>]_{mu,sigma}`` columns.

Every write, skip and log line follows /root/reference/rater.py:69-169:

* unsupported mode -> INFO log, nothing written;
* ``len(rosters) != 2`` (ERROR log) or any ``went_afk == 1`` (INFO log) ->
  ``trueskill_quality = 0`` and every ``any_afk = True``;
* otherwise two independent updates: the *shared* track (stored rating or a
  seed) and the *mode* track (stored, else the pre-update shared prior);
  quality is computed on the mode track (code wins over the comment at
  rater.py:140); ``trueskill_delta`` is the change of ``mu - sigma`` on the shared
  track, 0 for a first rating.  Writes happen participant by participant, so a
  player object repeated inside one match sees its own earlier write (exactly as
  the reference's loop does).

This is the per-match path used by the worker on CPU and as the semantic
reference for the batched MI355X path in :mod:`analyzer_amd.ops.rate`.
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

from ..config import MODES, RaterConfig
from ..utils.log import get_logger
from .tiers import seed_from_attributes
from .trueskill import TrueSkill

logger = get_logger()

MODE_COLUMN = {m: "trueskill_" + m for m in MODES}


def make_env(cfg: RaterConfig) -> TrueSkill:
    backend = "mpmath" if cfg.backend == "mpmath" else None
    if backend == "mpmath":
        import mpmath

        mpmath.mp.dps = 50  # reference precision (rater.py:8)
    return TrueSkill(backend=backend, mu=1500, sigma=1000, beta=cfg.beta,
                     tau=cfg.tau, draw_probability=0)


def trueskill_seed(player: Any, unknown_sigma: float) -> Tuple[float, float]:
    return seed_from_attributes(getattr(player, "rank_points_ranked", None),
                                getattr(player, "rank_points_blitz", None),
                                getattr(player, "skill_tier", None), unknown_sigma)


class MatchRater:
    """Stateless per-match rater bound to one TrueSkill environment."""

    def __init__(self, cfg: Optional[RaterConfig] = None, env: Optional[TrueSkill] = None):
        self.cfg = cfg or RaterConfig.from_env()
        self.env = env or make_env(self.cfg)

    # ---------------------------------------------------------------- helpers
    def seed(self, player: Any) -> Tuple[float, float]:
        return trueskill_seed(player, self.cfg.unknown_player_sigma)

    def _rate(self, teams: List[List[Tuple[float, float]]], ranks: List[int]):
        if self.cfg.backend == "closed":
            return self.env.rate_two_teams(teams[0], teams[1], ranks[0], ranks[1])
        env = self.env
        groups = [[env.create_rating(m, s) for m, s in t] for t in teams]
        return [[(float(r.mu), float(r.sigma)) for r in g] for g in env.rate(groups, ranks=ranks)]

    def _quality(self, teams: List[List[Tuple[float, float]]]) -> float:
        if self.cfg.backend == "closed":
            return self.env.quality_two_teams(teams[0], teams[1])
        env = self.env
        return float(env.quality([[env.create_rating(m, s) for m, s in t] for t in teams]))

    # ------------------------------------------------------------- the contract
    def rate_match(self, match: Any) -> None:
        column = MODE_COLUMN.get(match.game_mode)
        if column is None:
            logger.info("got unsupported game mode %s", match.game_mode)
            return

        any_afk = False
        if len(match.rosters) != 2:
            logger.error("got an invalid matchup %s", match.api_id)
            any_afk = True
        for participant in match.participants:
            participant.participant_items[0].any_afk = False
            if participant.went_afk == 1:
                logger.info("got an afk matchup %s", match.api_id)
                any_afk = True
                break
        if any_afk:
            match.trueskill_quality = 0
            for participant in match.participants:
                participant.participant_items[0].any_afk = True
            return

        shared_teams: List[List[Tuple[float, float]]] = []
        mode_teams: List[List[Tuple[float, float]]] = []
        for roster in match.rosters:
            t_shared, t_mode = [], []
            for participant in roster.participants:
                player = participant.player[0]
                if player.trueskill_mu is not None:
                    mu_s, sig_s = player.trueskill_mu, player.trueskill_sigma
                else:
                    mu_s, sig_s = self.seed(player)
                t_shared.append(_checked(mu_s, sig_s))
                mu_m = getattr(player, column + "_mu", None)
                if mu_m is not None:
                    sig_m = getattr(player, column + "_sigma")
                else:
                    mu_m, sig_m = mu_s, sig_s
                t_mode.append(_checked(mu_m, sig_m))
            shared_teams.append(t_shared)
            mode_teams.append(t_mode)

        logger.info("got a valid matchup %s", match.api_id)
        match.trueskill_quality = self._quality(mode_teams)

        ranks = [int(not r.winner) for r in match.rosters]
        for team, roster in zip(self._rate(shared_teams, ranks), match.rosters):
            for (mu, sigma), participant in zip(team, roster.participants):
                player = participant.player[0]
                if player.trueskill_mu is not None:
                    participant.trueskill_delta = (mu - sigma) - (
                        float(player.trueskill_mu) - float(player.trueskill_sigma))
                else:
                    participant.trueskill_delta = 0
                player.trueskill_mu = mu
                participant.trueskill_mu = mu
                player.trueskill_sigma = sigma
                participant.trueskill_sigma = sigma

        for team, roster in zip(self._rate(mode_teams, ranks), match.rosters):
            for (mu, sigma), participant in zip(team, roster.participants):
                player = participant.player[0]
                items = participant.participant_items[0]
                setattr(player, column + "_mu", mu)
                setattr(items, column + "_mu", mu)
                setattr(player, column + "_sigma", sigma)
                setattr(items, column + "_sigma", sigma)


def _checked(mu: Any, sigma: Any) -> Tuple[float, float]:
    mu_f, sig_f = float(mu), float(sigma)
    if sig_f == 0:
        raise ValueError("sigma**2 should be greater than 0")
    return mu_f, sig_f
