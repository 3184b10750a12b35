"""Shared helpers: run the per-object reference-semantics rater over a stream.

The object run applies /root/reference/rater.py semantics match by match, in
stream order, quarantining matches that raise (the batched engine reports them
with an error status and writes nothing), and rounds the stored ratings to fp32
after every match like the device roster does.
"""
from __future__ import annotations

import numpy as np
import torch

from analyzer_amd.config import MODES, TRACK_COLUMNS, RaterConfig
from analyzer_amd.models.match_rater import MatchRater
from analyzer_amd.ops import rate as R
from analyzer_amd.runtime.objects import matches_from_stream, players_from_roster


def _f32(x):
    return None if x is None else float(np.float32(x))


def object_run(roster, rec, K, cfg=None):
    cfg = cfg or RaterConfig()
    players = players_from_roster(roster.state, roster.attrs)
    matches = matches_from_stream(rec, K, players)
    rater = MatchRater(cfg)
    M, S = len(matches), 2 * K
    quality = np.full(M, np.nan)
    status = np.zeros(M, dtype=np.int64)
    outs = {k: np.full((M, S), np.nan) for k in ("s_mu", "s_sig", "delta", "m_mu", "m_sig")}
    for i, m in enumerate(matches):
        try:
            rater.rate_match(m)
        except KeyError:
            status[i] = R.ERR_SEED
            continue
        except ValueError as e:
            status[i] = R.ERR_EMPTY_ROSTER if "group" in str(e) else R.ERR_SIGMA
            continue
        if m.game_mode not in MODES:
            status[i] = R.UNSUPPORTED_MODE
            continue
        if len(m.rosters) != 2:
            status[i] = R.INVALID_ROSTERS
            quality[i] = m.trueskill_quality
            continue
        if any(p.participant_items[0].any_afk for p in m.participants):
            status[i] = R.AFK
            quality[i] = m.trueskill_quality
            continue
        quality[i] = m.trueskill_quality
        col = "trueskill_" + m.game_mode
        for ri, roster_obj in enumerate(m.rosters):
            for pos, p in enumerate(roster_obj.participants):
                j = ri * K + pos
                outs["s_mu"][i, j] = p.trueskill_mu
                outs["s_sig"][i, j] = p.trueskill_sigma
                outs["delta"][i, j] = p.trueskill_delta
                outs["m_mu"][i, j] = getattr(p.participant_items[0], col + "_mu")
                outs["m_sig"][i, j] = getattr(p.participant_items[0], col + "_sigma")
        for p in m.participants:  # fp32 storage like the device roster
            pl = p.player[0]
            for c in TRACK_COLUMNS:
                setattr(pl, c + "_mu", _f32(getattr(pl, c + "_mu")))
                setattr(pl, c + "_sigma", _f32(getattr(pl, c + "_sigma")))
    state = np.full((len(players), 8, 2), np.nan)
    for p, pl in enumerate(players):
        for t, c in enumerate(TRACK_COLUMNS):
            mu = getattr(pl, c + "_mu")
            if mu is not None:
                state[p, t, 0] = mu
                state[p, t, 1] = getattr(pl, c + "_sigma")
    return dict(quality=quality, status=status, state=state, **outs)


def assert_engine_matches(res: "R.RateResult", roster_after, ref, *, rtol, atol_mu, atol_delta):
    st = res.status.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(st, ref["status"])
    np.testing.assert_allclose(res.quality.cpu().numpy(), ref["quality"], rtol=rtol, atol=1e-6,
                               equal_nan=True)
    for k in ("s_mu", "s_sig", "m_mu", "m_sig"):
        np.testing.assert_allclose(getattr(res, k).cpu().numpy(), ref[k], rtol=rtol,
                                   atol=atol_mu, equal_nan=True, err_msg=k)
    np.testing.assert_allclose(res.delta.cpu().numpy(), ref["delta"], rtol=0, atol=atol_delta,
                               equal_nan=True)
    got = roster_after.tracks().cpu().numpy().astype(np.float64)
    got[:, 7] = np.nan  # spare granule
    exp = ref["state"].copy()
    np.testing.assert_allclose(got, exp, rtol=rtol, atol=atol_mu, equal_nan=True)


def status_of(res) -> dict:
    return res.status_counts()


def as_torch(x):
    return torch.as_tensor(x)


def _stateful_slots(rec: np.ndarray, K: int, P: int):
    """[M, 2K] bool: slots of matches that rate (the slots the schedule links) and
    [M, 2K] bool: the first slot of each distinct player of such a match."""
    S = 2 * K
    ids, m0, m1 = rec[:, :S], rec[:, S].astype(np.int64), rec[:, S + 1].astype(np.int64)
    n0, n1 = (m0 >> 8) & 0xFF, (m0 >> 16) & 0xFF
    pos = np.array([j if j < K else j - K for j in range(S)])
    inr = pos[None, :] < np.where(np.arange(S)[None, :] < K, n0[:, None], n1[:, None])
    bad = (n0 > K) | (n1 > K) | (inr & ((ids < 0) | (ids >= P))).any(1)
    rated = ((m0 & 0xFF) < 6) & ~bad & ((m0 >> 24) == 2) & (((m1 >> 2) & 1) == 0)
    slots = rated[:, None] & inr
    first = slots.copy()
    for j in range(S):
        for i in range(j):
            first[:, j] &= ~(slots[:, i] & (ids[:, i] == ids[:, j]))
    return slots, first
