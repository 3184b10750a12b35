#!/usr/bin/python3
"""Drop-in ``rater`` module: the reference's rater API on the new engine.

Same public names as /root/reference/rater.py (``UNKNOWN_PLAYER_SIGMA``,
``TAU``, ``vst_points``, ``env``, ``get_trueskill_seed``, ``rate_match``,
``InfoFilter``, ``logger``), so code and tests written against the reference
import this module unchanged.  The work is done by
:class:`analyzer_amd.models.match_rater.MatchRater` (exact two-team closed form
in fp64 by default; ``RATER_BACKEND=ep`` runs the general factor graph and
``RATER_BACKEND=mpmath`` the 50-digit factor graph the reference uses).
For millions of matches use the batched MI355X path in
:mod:`analyzer_amd.ops.rate` instead of this per-object API.
"""
from analyzer_amd.config import RaterConfig
from analyzer_amd.models.match_rater import MatchRater
from analyzer_amd.models.tiers import vst_points  # noqa: F401  (public name)
from analyzer_amd.utils.log import InfoFilter, get_logger  # noqa: F401

_cfg = RaterConfig.from_env()
UNKNOWN_PLAYER_SIGMA = _cfg.unknown_player_sigma
TAU = _cfg.tau

_rater = MatchRater(_cfg)
env = _rater.env
logger = get_logger()


def get_trueskill_seed(player):
    """Return a (mu, sigma) based on information known about a player."""
    return _rater.seed(player)


def rate_match(match):
    """Mutate a match structure by updating TrueSkill values (returns None)."""
    return _rater.rate_match(match)
