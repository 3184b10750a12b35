"""Skill-tier -> rank-point table and rating seeds.

The reference builds ``vst_points`` for tiers -1..29 as a piecewise-linear
ladder (/root/reference/rater.py:13-27); tier 30 is absent there, so a tier-30
(or tier ``None``) player with no rank points raises ``KeyError`` when seeded
(/root/reference/rater.py:60).  We keep that table exactly, and expose the
same data as a dense array for the device-side seed in csrc/rate_kernels.hip.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

TIER_MIN = -1
TIER_MAX = 29  # inclusive; 30 deliberately missing (reference behaviour)


def _build_vst_points() -> Dict[int, float]:
    # (first tier of segment, last tier of segment, step)
    pts: Dict[int, float] = {-1: 1, 0: 1}
    segments = ((1, 11, 109 + 1 / 11), (12, 15, 50.0), (16, 24, 66 + 2 / 3),
                (25, 27, 133 + 1 / 3), (28, 29, 200.0))
    anchor = 0.0
    for first, last, step in segments:
        for tier in range(first, last + 1):
            # every tier sits half a step past the segment anchor
            pts[tier] = anchor + step * (tier - first + 1.5)
        anchor = pts[last]
    return pts


vst_points: Dict[int, float] = _build_vst_points()


def vst_table() -> list:
    """Dense table indexed by ``tier + 1`` for tiers -1..29 (length 31)."""
    return [float(vst_points[t]) for t in range(TIER_MIN, TIER_MAX + 1)]


def seed_from_attributes(rank_points_ranked: Optional[float], rank_points_blitz: Optional[float],
                         skill_tier: Optional[int], unknown_sigma: float) -> Tuple[float, float]:
    """(mu, sigma) seed for a player with no shared rating.

    Same decision procedure as /root/reference/rater.py:42-62: the larger of the
    non-null, non-zero rank-point columns seeds with sigma = 2/3 of
    ``unknown_sigma``; otherwise the tier table seeds with the full
    ``unknown_sigma``.  Missing tier entries raise ``KeyError``.
    """
    rp = None
    for cand in (rank_points_ranked, rank_points_blitz):
        if cand is not None and cand == cand and cand != 0 and (rp is None or cand > rp):
            rp = cand
    if rp is not None:
        sigma = unknown_sigma * (2.0 / 3.0)
        return float(rp) + sigma, sigma
    sigma = unknown_sigma
    return vst_points[skill_tier] + sigma, sigma
