"""Rate a batch of ORM/POPO matches with the batched engine (worker ``ENGINE=native``).

The reference rates a batch by calling ``rater.rate_match`` on every match in
``created_at`` order (/root/reference/worker.py:176-192).  This path encodes
the batch once into the device stream layout (objects.encode_matches), builds
a roster of the batch's distinct players (one object = one row, so a player
met twice in the batch is rated sequentially, as in the reference), runs the
exact dataflow engine (MI355X kernels on a GPU, C++ fp64 host mirror on the
CPU), and writes the results back onto the same attributes the reference
writes (rater.py:103-105,141,151-169):

* unsupported mode: nothing;
* AFK / not two rosters: ``trueskill_quality = 0`` and every ``any_afk = True``;
* rated: quality, per-participant shared (mu, sigma, delta), per-item mode
  (mu, sigma), ``any_afk = False``, and the players' final shared + mode ratings;
* error classes (the reference raises: tier None/30, sigma 0, empty roster,
  non-finite result): nothing is written and the match is reported so the
  worker can quarantine it or fail the batch.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from ..config import MODES, TRACK_COLUMNS
from ..ops import rate as R
from .objects import (STAT_COLUMNS, Match, ParticipantStats, Player, encode_matches,
                      roster_from_players)

MAX_TEAM = 5  # kernel instantiations: K = 1..5


def team_size(matches: Sequence[Match]) -> int:
    k = 1
    for m in matches:
        for r in list(m.rosters)[:2]:
            k = max(k, len(r.participants))
    return k


def _f(x: float) -> Optional[float]:
    x = float(x)
    return None if math.isnan(x) else x


class ObjectBatchRater:
    """Batched rating of object matches; results written back in place."""

    def __init__(self, rater: Optional[R.BatchRater] = None, device: Optional[str] = None):
        self.rater = rater or R.BatchRater()
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)

    def supports(self, matches: Sequence[Match]) -> bool:
        return team_size(matches) <= MAX_TEAM

    def rate(self, matches: Sequence[Match], telemetry=None) -> List[int]:
        """Rate ``matches`` (already in chronological order); returns the status per match.

        ``telemetry``: a ``TelemetrySpec`` -- synthetic per-event telemetry of the
        batch is aggregated in the same launch (K8 fused streaming mode) and
        written to ``participant.participant_stats[0]``."""
        if not matches:
            return []
        K = team_size(matches)
        if K > MAX_TEAM:
            raise ValueError("teams of %d players exceed the batched engine (max %d)" % (K, MAX_TEAM))
        players, index = [], {}
        for m in matches:
            for r in list(m.rosters)[:2]:
                for p in r.participants:
                    pl = p.player[0]
                    if id(pl) not in index:
                        index[id(pl)] = len(players)
                        players.append(pl)
        # (a batch without participants still needs one roster row to launch)
        roster = roster_from_players(players or [Player("")], device=self.device)
        rec = encode_matches(matches, index, K, device=self.device)
        tele = stats = None
        if telemetry is not None:
            from ..ops.telemetry import allocate_stats, make_telemetry
            tel = make_telemetry(telemetry, rec, K, ids=[m.api_id for m in matches])
            stats = allocate_stats(len(matches), K, self.device)
            tele = (tel.evoff, tel.events, stats)
        res = self.rater.rate(roster, rec, K, telemetry=tele)
        self._write_back(matches, res, roster, players, K)
        status = [int(s) for s in res.status.cpu().tolist()]
        if stats is not None:
            self._write_stats(matches, stats, K, status)
        return status

    @staticmethod
    def _write_stats(matches, stats: torch.Tensor, K: int, status) -> None:
        """participant_stats of every committed match (not the quarantined ones)."""
        st = stats.cpu().double().numpy()
        bad = set(R.ERROR_STATUSES) | {R.NOT_PROCESSED}
        for i, m in enumerate(matches):
            if status[i] in bad:
                continue
            for ri, r in enumerate(list(m.rosters)[:2]):
                for pos, p in enumerate(r.participants[:K]):
                    vals = dict(zip(STAT_COLUMNS, (float(v) for v in st[i, ri * K + pos])))
                    p.participant_stats = [ParticipantStats(p.api_id, **vals)]

    def _write_back(self, matches, res: R.RateResult, roster, players, K: int) -> None:
        st = res.status.cpu().numpy()
        q = res.quality.cpu().double().numpy()
        s_mu, s_sig, dl = (t.cpu().double().numpy() for t in (res.s_mu, res.s_sig, res.delta))
        m_mu, m_sig = (t.cpu().double().numpy() for t in (res.m_mu, res.m_sig))
        final = roster.state.cpu().double().numpy() if players else None
        touched: Dict[int, set] = {}
        for i, m in enumerate(matches):
            s = int(st[i])
            if s == R.UNSUPPORTED_MODE or s in R.ERROR_STATUSES or s == R.NOT_PROCESSED:
                continue
            if s in (R.AFK, R.INVALID_ROSTERS):
                m.trueskill_quality = 0
                for p in m.participants:
                    p.participant_items[0].any_afk = True
                continue
            mode = MODES.index(m.game_mode)
            col = TRACK_COLUMNS[1 + mode]
            m.trueskill_quality = float(q[i])
            for p in m.participants:
                p.participant_items[0].any_afk = False
            for ri, r in enumerate(list(m.rosters)[:2]):
                for pos, p in enumerate(r.participants):
                    j = ri * K + pos
                    p.trueskill_mu = float(s_mu[i, j])
                    p.trueskill_sigma = float(s_sig[i, j])
                    p.trueskill_delta = float(dl[i, j])
                    it = p.participant_items[0]
                    setattr(it, col + "_mu", float(m_mu[i, j]))
                    setattr(it, col + "_sigma", float(m_sig[i, j]))
                    touched.setdefault(id(p.player[0]), set()).update((0, 1 + mode))
        if final is None:
            return
        for row, pl in enumerate(players):
            for t in sorted(touched.get(id(pl), ())):
                col = TRACK_COLUMNS[t]
                setattr(pl, col + "_mu", _f(final[row, 4 * t]))
                setattr(pl, col + "_sigma", _f(final[row, 4 * t + 2]))
