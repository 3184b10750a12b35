"""Plain-Python match objects and tensor <-> object converters.

The object shapes follow the attribute names the reference reads and writes
(SURVEY §2.1 data-model table; /root/reference/worker.py:43-83 relationships,
all list-valued: ``participant.player[0]``, ``participant.participant_items[0]``).
They serve three purposes:

* the in-memory store of the worker (no MySQL in this environment);
* encoding a batch of ORM/POPO matches into the device stream layout and
  writing the kernel outputs back onto the objects (the worker's native path);
* cross-checking the batched engine against the per-object rater.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from ..config import MODES, N_TRACKS, TRACK_COLUMNS

MODE_INDEX = {m: k for k, m in enumerate(MODES)}


def _none_if_nan(x: float) -> Optional[float]:
    return None if x is None or (isinstance(x, float) and math.isnan(x)) else x


class Player:
    def __init__(self, api_id: str = "", skill_tier=None, rank_points_ranked=None,
                 rank_points_blitz=None, **ratings):
        self.api_id = api_id
        self.skill_tier = skill_tier
        self.rank_points_ranked = rank_points_ranked
        self.rank_points_blitz = rank_points_blitz
        for col in TRACK_COLUMNS:
            setattr(self, col + "_mu", ratings.get(col + "_mu"))
            setattr(self, col + "_sigma", ratings.get(col + "_sigma"))


class ParticipantItems:
    def __init__(self, api_id: str = ""):
        self.api_id = api_id
        self.any_afk = False
        for col in TRACK_COLUMNS[1:]:
            setattr(self, col + "_mu", None)
            setattr(self, col + "_sigma", None)


STAT_COLUMNS = ("kills", "deaths", "assists", "damage", "gold", "farm", "healing", "events")


class ParticipantStats:
    """``participant_stats`` row (mapped but never filled by the reference,
    worker.py:75-78; here filled by the K8 telemetry aggregation)."""

    def __init__(self, api_id: str = "", **values):
        self.api_id = api_id
        for c in STAT_COLUMNS:
            setattr(self, c, values.get(c))


class Participant:
    def __init__(self, player: Player, api_id: str = "", went_afk=0, skill_tier=None,
                 items: Optional[ParticipantItems] = None):
        self.api_id = api_id
        self.player_api_id = player.api_id
        self.went_afk = went_afk
        self.skill_tier = skill_tier
        self.trueskill_mu = None
        self.trueskill_sigma = None
        self.trueskill_delta = None
        self.player = [player]
        self.participant_items = [items or ParticipantItems(api_id)]
        self.participant_stats: List[ParticipantStats] = []


class Roster:
    def __init__(self, participants: List[Participant], winner=None, api_id: str = ""):
        self.api_id = api_id
        self.winner = winner
        self.participants = participants


class Match:
    def __init__(self, game_mode: str, rosters: List[Roster], api_id: str = "",
                 created_at: float = 0.0):
        self.api_id = api_id
        self.game_mode = game_mode
        self.created_at = created_at
        self.rosters = rosters
        self.participants = [p for r in rosters for p in r.participants]
        self.trueskill_quality = None


# ------------------------------------------------------------------ tensors -> objects
def players_from_roster(state: torch.Tensor, attrs: torch.Tensor) -> List[Player]:
    st = state.detach().cpu().double().numpy()
    at = attrs.detach().cpu().double().numpy()
    players = []
    for p in range(st.shape[0]):
        kw = {}
        for t, col in enumerate(TRACK_COLUMNS):
            kw[col + "_mu"] = _none_if_nan(float(st[p, 4 * t]))
            kw[col + "_sigma"] = _none_if_nan(float(st[p, 4 * t + 2])) if kw[col + "_mu"] is not None else None
        tier = _none_if_nan(float(at[p, 2]))
        players.append(Player("p%d" % p, None if tier is None else int(tier),
                              _none_if_nan(float(at[p, 0])), _none_if_nan(float(at[p, 1])), **kw))
    return players


def matches_from_stream(rec: torch.Tensor, K: int, players: Sequence[Player], base: int = 0,
                        prefix: str = "m") -> List[Match]:
    """Decode stream records into objects (invalid records -> nrosters padding).
    Match ``i`` gets api id ``<prefix><base+i>`` and ``created_at = base + i``."""
    r = rec.detach().cpu().numpy()
    S = 2 * K
    out = []
    for m in range(r.shape[0]):
        g = base + m
        m0, m1 = int(r[m, S]) & 0xffffffff, int(r[m, S + 1]) & 0xffffffff
        mode = m0 & 0xff
        n0, n1, nrost = (m0 >> 8) & 0xff, (m0 >> 16) & 0xff, (m0 >> 24) & 0xff
        afk_mask = (m1 >> 8) & 0xffffff
        rosters = []
        k = 0
        for ri, n in enumerate((n0, n1)):
            parts = []
            for pos in range(n):
                pid = int(r[m, ri * K + pos])
                afk = 1 if (afk_mask >> k) & 1 else 0
                parts.append(Participant(players[pid], "%s%dp%d" % (prefix, g, k), went_afk=afk))
                k += 1
            winner = bool(m1 & (1 << ri))
            rosters.append(Roster(parts, winner=winner, api_id="%s%dr%d" % (prefix, g, ri)))
        for extra in range(max(0, nrost - 2)):
            rosters.append(Roster([], winner=False, api_id="%s%dx%d" % (prefix, g, extra)))
        if nrost < 2:
            rosters = rosters[:nrost]
        game_mode = MODES[mode] if mode < len(MODES) else "private"
        out.append(Match(game_mode, rosters, api_id="%s%d" % (prefix, g), created_at=float(g)))
    return out


# ------------------------------------------------------------------ objects -> tensors
def roster_from_players(players: Sequence[Player], device="cpu"):
    from ..ops.rate import Roster as TRoster

    P = len(players)
    state = torch.zeros((P, 32), dtype=torch.float64)
    state[:, 0::2] = float("nan")
    attrs = torch.full((P, 4), float("nan"), dtype=torch.float64)
    attrs[:, 3] = 0
    for p, pl in enumerate(players):
        for t, col in enumerate(TRACK_COLUMNS):
            mu = getattr(pl, col + "_mu", None)
            if mu is not None:
                state[p, 4 * t] = float(mu)
                sig = getattr(pl, col + "_sigma", None)
                state[p, 4 * t + 2] = float(sig) if sig is not None else float("nan")
        for c, name in enumerate(("rank_points_ranked", "rank_points_blitz", "skill_tier")):
            v = getattr(pl, name, None)
            if v is not None:
                attrs[p, c] = float(v)
    return TRoster(state.float().to(device), attrs.float().to(device), epoch=0)


def encode_matches(matches: Sequence[Match], player_index: Dict[int, int], K: int,
                   device="cpu") -> torch.Tensor:
    """Encode ORM/POPO matches into ``[M, 2K+2]`` records.

    ``player_index`` maps ``id(player_object)`` -> roster row.  Rosters beyond
    the second only count towards ``nrosters`` (the reference marks such
    matches invalid before touching players).
    """
    S = 2 * K
    rec = torch.full((len(matches), S + 2), -1, dtype=torch.int32)
    for m, match in enumerate(matches):
        mode = MODE_INDEX.get(match.game_mode, 255)
        rosters = list(match.rosters)
        ns = [len(r.participants) for r in rosters[:2]] + [0, 0]
        afk_mask = 0
        k = 0
        for ri, roster in enumerate(rosters[:2]):
            for pos, part in enumerate(roster.participants):
                if pos < K:
                    rec[m, ri * K + pos] = player_index[id(part.player[0])]
                if part.went_afk == 1:
                    afk_mask |= 1 << min(k, 23)
                k += 1
        # participants outside the first two rosters can also be AFK
        for roster in rosters[2:]:
            for part in roster.participants:
                if part.went_afk == 1:
                    afk_mask |= 1 << 23
        w0 = bool(rosters[0].winner) if len(rosters) > 0 else False
        w1 = bool(rosters[1].winner) if len(rosters) > 1 else False
        n0 = min(ns[0], 255)
        n1 = min(ns[1], 255)
        m0 = (mode & 0xff) | (n0 << 8) | (n1 << 16) | (min(len(rosters), 255) << 24)
        m1 = (1 if w0 else 0) | (2 if w1 else 0) | (4 if afk_mask else 0) | ((afk_mask & 0xffffff) << 8)
        rec[m, S] = m0 - (1 << 32) if m0 >= (1 << 31) else m0
        rec[m, S + 1] = m1 - (1 << 32) if m1 >= (1 << 31) else m1
    return rec.to(device)
