"""Exact data-parallel rating by conflict-free rounds.

A CORRECTNESS ORACLE, not a scaling mode: no bench / worker / re-rate path selects it.
Depth x exchange latency bounds any exact multi-GPU mode above one GPU rating the
window alone (docs/EXACT_MULTI_GPU.md: 7.26 s vs 3.8 ms on a 1M-match window).

Exact chronological semantics (/root/reference/worker.py:176,191-192) allow
parallelism only between matches that share no player.  The levelizer (K5: on
the device a dataflow over the rating's own schedule, csrc/levels.hip; on the
host a C++ walk) gives every match its round: 1 + the latest round of any of its
players, 0 for matches that touch no state (they go with round 1).
Matches of one round are disjoint, so ranks split each round into contiguous
slices, rate their slice against their replica, and exchange ONLY the rows
they changed.  The result is bit-identical to one process rating the window in
order (ratings; the tag words of exchanged rows are reset).

Everything about the window's shape is known on the host before the first
launch -- rounds, slice bounds, the largest slice -- so the round loop never
waits for the device: a rank's slices are gathered once into round order, and
per round it launches the rating, one pack kernel (csrc/sweep.hip: the rows of
its rated players + their ids, -1 padded to the round's largest slice, which
every rank reads off the shared plan), ONE ``all_gather_into_tensor`` and one
unpack kernel.  No ``.item()``, no size exchange.

How far this scales is set by the DAG, not by the implementation: a 10M 3v3
window over 1M uniform players has ~900 rounds of ~11k matches, so exact DP
needs ~900 exchanges per window.  Grouping g rounds per exchange stays exact
only if no dependency crosses ranks inside the group, i.e. if whole connected
components of the g-round sub-DAG go to one rank; a player there has
~0.066 g occurrences, so at 5 x 0.066 g > 1 (g > 3) a giant component forms and
grouping stops paying.  Exact mode is therefore the way to spread one window's
outputs over several devices; throughput scaling is sweep DP
(parallel/sweep.py), whose causal re-sweeps reach exact results with
``sweeps == world`` in ``2 * world`` collectives (at ``world``x the rating work).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..config import EngineConfig
from ..ops.native import native
from ..ops.rate import BatchRater, RateResult, Roster
from .comm import world


def rounds(rec: torch.Tensor, K: int, num_players: int, rater: Optional[BatchRater] = None):
    """(level per match [M] int32 on the host, number of rounds).

    A device stream is levelized on the device (csrc/levels.hip: a dataflow over
    the same radix schedule the rating uses, milliseconds per 10M-match window);
    a host stream by the sequential C++ walk (host.cpp levels_k).  Both give the
    same levels (tests/test_engine_gpu.py)."""
    if rec.is_cuda:
        sched = (rater or BatchRater()).schedule(rec, K, num_players, tag="_levels")
        level, depth = native().levels_device(rec.contiguous(), K, num_players, sched.link, sched.deps)
        return level.cpu(), int(depth)
    level, depth = native().levels(rec.detach().cpu().contiguous(), K, num_players)
    return level, int(depth)


class RoundPlan:
    """Host-side plan of a window: round order, per-rank slice bounds, capacity."""

    def __init__(self, level: torch.Tensor, size: int):
        lv = np.maximum(level.numpy().astype(np.int64), 1)  # stateless matches go with round 1
        M = lv.size
        self.order = np.argsort(lv, kind="stable")             # round order, stable in time
        counts = np.bincount(lv, minlength=int(lv.max()) + 1 if M else 2)[1:]
        self.n_rounds = int(counts.size)
        starts = np.concatenate([[0], np.cumsum(counts)])
        # slice q of round r: [starts[r] + r_q, starts[r] + r_{q+1}) with sizes differing by <= 1
        q = np.arange(size + 1)
        self.bounds = starts[:-1, None] + (counts[:, None] * q[None, :]) // size   # [R, size+1]
        sizes = self.bounds[:, 1:] - self.bounds[:, :-1]
        self.max_slice = int(sizes.max()) if M else 0
        # per round: the largest slice of any rank -- the round's exchange size
        # (every rank knows the plan, so the gathers agree without a size exchange)
        self.round_max = sizes.max(1).astype(np.int64) if M else np.zeros(0, np.int64)


def check_rounds(rec: torch.Tensor, K: int, plan: "RoundPlan", num_players: int) -> int:
    """Race detector: the first round whose matches share a player, or
    -1.  One kernel per round claims every rated slot's player for its match in a
    64-bit owner table (csrc/sweep.hip check_round_kernel); a second claim by
    another match of the same round raises the flag."""
    dev = rec.device
    owner = torch.zeros(max(num_players, 1), dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    order = torch.from_numpy(plan.order).to(dev)
    for r in range(plan.n_rounds):
        lo, hi = int(plan.bounds[r, 0]), int(plan.bounds[r, -1])
        native().check_round(rec, K, order[lo:hi], r, owner, flag)
        if rec.device.type == "cpu" and int(flag[0]):
            return r
    if int(flag[0]):  # device: one sync at the end; find the round on the host
        return check_rounds(rec.cpu(), K, plan, num_players)
    return -1


def rate_exact_dp(rater: BatchRater, roster: Roster, rec: torch.Tensor, K: int,
                  group=None, level: Optional[torch.Tensor] = None) -> RateResult:
    """Rate ``rec`` exactly across the ranks of ``group`` (replicated roster).

    Every rank returns the full-window outputs for the matches IT rated and
    NaN / status 255 elsewhere (outputs stay sharded; gather them if needed)."""
    rank, size = world(group)
    M = rec.shape[0]
    dev = roster.device
    out = RateResult.allocate(M, K, dev)
    out.packed.fill_(float("nan"))
    out.status.fill_(255)
    if M == 0:
        return out
    if level is None:
        level, _ = rounds(rec.to(dev) if dev.type == "cuda" else rec, K, roster.num_players, rater)
    plan = RoundPlan(level, size)
    if EngineConfig.from_env().check_rounds:
        bad = check_rounds(rec, K, plan, roster.num_players)
        if bad >= 0:
            raise RuntimeError("exact DP: round %d has two matches sharing a player" % bad)
    S = 2 * K
    # this rank's matches, in round order, gathered once
    mine = np.concatenate([np.arange(plan.bounds[r, rank], plan.bounds[r, rank + 1])
                           for r in range(plan.n_rounds)]).astype(np.int64)
    idx = torch.from_numpy(plan.order[mine]).to(dev)
    my_rec = rec.index_select(0, idx) if rec.device == dev else rec.index_select(0, idx.cpu()).to(dev)
    my_out = RateResult.allocate(int(idx.numel()), K, dev)
    offs = np.concatenate([[0], np.cumsum(plan.bounds[:, rank + 1] - plan.bounds[:, rank])])
    cap = max(1, plan.max_slice * S)
    f = dict(dtype=torch.float32, device=dev)
    send_buf = torch.empty((cap, 33), **f)
    recv_buf = torch.empty((size * cap, 33), **f)
    staged = dev.type == "cuda" and size > 1 and dist.get_backend(group) == "gloo"
    if dev.type == "cuda":
        rater.clear_sticky(dev)
    for r in range(plan.n_rounds):
        lo, hi = int(offs[r]), int(offs[r + 1])
        if hi > lo:
            sub = my_rec[lo:hi]
            res = rater.rate(roster, sub, K, out=RateResult(
                my_out.quality[lo:hi], my_out.status[lo:hi], my_out.s_mu[lo:hi], my_out.s_sig[lo:hi],
                my_out.delta[lo:hi], my_out.m_mu[lo:hi], my_out.m_sig[lo:hi],
                packed=my_out.packed[lo:hi]), check=False)
        if size <= 1:
            continue
        # this round's exchange: the largest slice's rows (a 10M window's rounds
        # average ~1/20 of the largest), not the window-wide capacity
        rc = max(1, int(plan.round_max[r]) * S)
        send, recv = send_buf[:rc], recv_buf[:size * rc]
        if hi > lo:
            native().pack_rows(sub, K, res.status, roster.state, send)
        else:
            send[:, 32].view(torch.int32).fill_(-1)
        if staged:  # gloo moves host memory only
            h = torch.empty((size * rc, 33))
            dist.all_gather_into_tensor(h, send.cpu(), group=group)
            recv.copy_(h)
        else:
            dist.all_gather_into_tensor(recv, send, group=group)
        # every rank's changed rows (this rank's own are rewritten unchanged, tags reset)
        native().unpack_rows(recv, roster.state)
    roster.epoch = None  # foreign rows carry reset tags; re-zero before the next eager launch
    if dev.type == "cuda":
        rater.check_errors(dev, sticky=True)  # every round's launch, one sync
    # scatter this rank's outputs back to window order
    out.packed.index_copy_(0, idx, my_out.packed)
    return out
