"""Exact data-parallel rating by conflict-free rounds.

Exact chronological semantics (/root/reference/worker.py:176,191-192) allow
parallelism only between matches that share no player.  The host levelizer
(K5, ``native().levels``) assigns every match its round: 1 + the latest round
of any of its players.  Matches of one round are disjoint, so ranks split each
round, rate their share against their replica, and exchange ONLY the rows they
changed: one variable-size all-gather of (player id, 128-B row) per round.
The result is bit-identical to one process rating the window in order.

This mode is latency-bound -- one collective per round, ~900 rounds for a 10M
3v3 window over 1M players -- which is why the throughput path on one node is
the single-GPU dataflow engine plus the sweep merge (parallel/sweep.py); exact
DP is the correctness-preserving way to spread one window over several
devices (e.g. when its outputs do not fit one GPU).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops.native import native
from ..ops.rate import BatchRater, RateResult, Roster
from .comm import world


def rounds(rec: torch.Tensor, K: int, num_players: int):
    """(level per match [M] int32 on the host, number of rounds)."""
    level, depth = native().levels(rec.detach().cpu().contiguous(), K, num_players)
    return level, int(depth)


def _gather_rows(ids: torch.Tensor, rows: torch.Tensor, group=None):
    """All-gather variable-size (ids, rows) from every rank (padded to the max)."""
    _, size = world()
    n = torch.tensor([ids.numel()], dtype=torch.int64, device=ids.device)
    sizes = [torch.zeros_like(n) for _ in range(size)]
    dist.all_gather(sizes, n, group=group)
    cap = int(max(int(s.item()) for s in sizes))
    if cap == 0:
        return [], []
    pid = torch.full((cap,), -1, dtype=ids.dtype, device=ids.device)
    pid[:ids.numel()] = ids
    prow = torch.zeros((cap, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    prow[:rows.shape[0]] = rows
    all_ids = [torch.empty_like(pid) for _ in range(size)]
    all_rows = [torch.empty_like(prow) for _ in range(size)]
    dist.all_gather(all_ids, pid, group=group)
    dist.all_gather(all_rows, prow, group=group)
    return ([a[:int(s.item())] for a, s in zip(all_ids, sizes)],
            [r[:int(s.item())] for r, s in zip(all_rows, sizes)])


def rate_exact_dp(rater: BatchRater, roster: Roster, rec: torch.Tensor, K: int,
                  group=None, level: Optional[torch.Tensor] = None) -> RateResult:
    """Rate ``rec`` exactly across the ranks of ``group`` (replicated roster).

    Every rank returns the full-window outputs for the matches IT rated and
    NaN / status 255 elsewhere (outputs stay sharded; gather them if needed)."""
    rank, size = world()
    M = rec.shape[0]
    dev = roster.device
    out = RateResult.allocate(M, K, dev)
    out.quality.fill_(float("nan"))
    out.status.fill_(255)
    for t in (out.s_mu, out.s_sig, out.delta, out.m_mu, out.m_sig):
        t.fill_(float("nan"))
    if level is None:
        level, _ = rounds(rec, K, roster.num_players)
    level = level.to(torch.int64)
    # stateless matches (level 0) go with round 1; ranks take every size-th match of a round
    order = torch.argsort(level.clamp(min=1) * (M + 1) + torch.arange(M), stable=True)
    lv = level.clamp(min=1)[order]
    bounds = torch.searchsorted(lv, torch.arange(1, int(lv.max().item()) + 2 if M else 2))
    S = 2 * K
    for r in range(len(bounds) - 1):
        idx = order[int(bounds[r]):int(bounds[r + 1])]
        mine = idx[rank::size]
        if mine.numel():
            mine_d = mine.to(dev)
            sub = rec.index_select(0, mine_d) if rec.device == dev else rec.index_select(0, mine).to(dev)
            res = rater.rate(roster, sub, K)
            out.quality[mine_d] = res.quality
            out.status[mine_d] = res.status
            for a, b in ((out.s_mu, res.s_mu), (out.s_sig, res.s_sig), (out.delta, res.delta),
                         (out.m_mu, res.m_mu), (out.m_sig, res.m_sig)):
                a[mine_d] = b
            # only rated matches change rows; the players of stateless matches (AFK,
            # unsupported, errors) may be updated by another rank in this round
            ids = sub[res.status == 0][:, :S].reshape(-1)
            ids = torch.unique(ids[ids >= 0])
        else:
            ids = torch.empty(0, dtype=torch.int32, device=dev)
        if size > 1:
            all_ids, all_rows = _gather_rows(ids.to(torch.int64), roster.state.index_select(0, ids.long()),
                                             group)
            for q, (i, rw) in enumerate(zip(all_ids, all_rows)):
                if q != rank and i.numel():
                    roster.state[i] = rw
    return out
