"""Synthetic rosters and match streams (BASELINE "synthetic" data).

The reference reads players/matches from MySQL and match ids from RabbitMQ
(/root/reference/worker.py:38-101).  For benchmarks and tests the engine
generates both on the device with a counter-based RNG instead; the same
generator runs in the C++ host mirror, bit-identically, so CPU tests and GPU
runs see the same data for the same seed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from ..config import MODES
from .native import native

U32 = 1 << 32


def prob_u32(p: float) -> int:
    """Quantise a probability to the uint32 threshold the kernels compare against."""
    return int(min(max(round(float(p) * U32), 0), U32 - 1))


@dataclass(frozen=True)
class RosterSpec:
    num_players: int = 1_000_000
    seed: int = 1
    p_tier_null: float = 0.0       # skill_tier NULL
    p_tier_bad: float = 0.0        # skill_tier 30 (no vst_points entry)
    p_rp_ranked: float = 0.30      # rank_points_ranked present
    p_rp_blitz: float = 0.15       # rank_points_blitz present
    p_rated: float = 0.50          # player already has a shared TrueSkill
    p_mode_rated: float = 0.50     # ... and each mode track
    mu_lo: float = 1000.0
    mu_span: float = 1500.0
    sig_lo: float = 80.0
    sig_span: float = 300.0


@dataclass(frozen=True)
class StreamSpec:
    team_size: int = 3
    seed: int = 2
    modes: Dict[str, float] = field(default_factory=lambda: {
        "casual": 0.35, "ranked": 0.40, "blitz": 0.15, "br": 0.10})
    p_unsupported: float = 0.0     # e.g. "private" lobbies the rater skips
    p_uneven: float = 0.0          # roster 1 one player short
    p_bad_rosters: float = 0.0     # three rosters -> invalid matchup
    p_tie: float = 0.01            # both rosters winner=False
    p_afk: float = 0.02            # somebody went AFK
    p_hot: float = 0.0             # probability a slot draws from the hot set
    hot_fraction: float = 0.01     # hot set = first fraction of the roster
    skew: int = 1                  # power-law activity: player = floor(u^skew * P) (1 = uniform)

    def mode_cdf(self):
        weights = [float(self.modes.get(m, 0.0)) for m in MODES]
        total = sum(weights) + float(self.p_unsupported)
        if total <= 0:
            raise ValueError("stream spec has no game modes")
        cdf, acc = [], 0.0
        for w in weights:
            acc += w / total
            cdf.append(prob_u32(acc))
        cdf.append(U32 - 1)
        return cdf


def make_roster(spec: RosterSpec, device="cpu"):
    """Return a :class:`Roster` (state [P,32] f32, attrs [P,4] f32) for ``spec``."""
    from .rate import Roster

    P = int(spec.num_players)
    state = torch.empty((P, 32), dtype=torch.float32, device=device)
    attrs = torch.empty((P, 4), dtype=torch.float32, device=device)
    native().gen_roster(state, attrs, int(spec.seed), prob_u32(spec.p_tier_null),
                        prob_u32(spec.p_tier_bad), prob_u32(spec.p_rp_ranked),
                        prob_u32(spec.p_rp_blitz), prob_u32(spec.p_rated),
                        prob_u32(spec.p_mode_rated), spec.mu_lo, spec.mu_span, spec.sig_lo,
                        spec.sig_span)
    return Roster(state, attrs, epoch=0)


def make_stream(spec: StreamSpec, num_matches: int, num_players: int, K: Optional[int] = None,
                base: int = 0, device="cpu", out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Generate ``num_matches`` records ``[M, 2K+2]`` int32 (layout: csrc/common.h).

    ``base`` is the global index of the first match, so consecutive windows or
    per-rank shards of one logical stream are produced independently.
    """
    K = int(K or spec.team_size)
    if out is None:
        out = torch.empty((int(num_matches), 2 * K + 2), dtype=torch.int32, device=device)
    hot = max(1, int(round(spec.hot_fraction * num_players)))
    native().gen_stream(out, K, int(spec.seed), int(base), int(num_players), int(spec.team_size),
                        spec.mode_cdf(), prob_u32(spec.p_uneven), prob_u32(spec.p_bad_rosters),
                        prob_u32(spec.p_tie), prob_u32(spec.p_afk), prob_u32(spec.p_hot),
                        min(hot, num_players), int(spec.skew))
    return out
