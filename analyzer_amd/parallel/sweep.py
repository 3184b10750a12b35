"""Data-parallel rating with per-window posterior merge.

Each rank holds a replica of the roster (128 B/player: 1M players = 128 MB, so
replication is the right call on 288 GB devices), rates its shard of every
window exactly and in order, and then all ranks merge what they learned with
ONE dense all-reduce of natural-parameter messages (csrc/sweep.hip):

    begin(roster)   -> snapshot the window-start roster
    <rate the local shard exactly>
    merge(roster)   -> messages against a common base -> all_reduce(SUM) over
                       RCCL/xGMI -> apply (csrc/sweep_core.h)

With one rank the merge is skipped (the exact single-GPU result stands).
Backend: ``nccl`` (RCCL on ROCm) for device tensors, ``gloo`` for CPU tests.
The reference has no counterpart: horizontal scale-out there is N worker
replicas racing on MySQL rows (/root/reference/worker.py:91,174-194).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..config import RaterConfig
from ..models.tiers import vst_table
from ..ops.native import native

MAX_RANKS = 15  # touch counts are base-16 fields in fp32 (see csrc/sweep_core.h)


class SweepMerger:
    def __init__(self, num_players: int, device, cfg: Optional[RaterConfig] = None,
                 group=None, comm_dtype: str = "fp32"):
        self.P = int(num_players)
        self.device = torch.device(device)
        self.cfg = cfg or RaterConfig.from_env()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > MAX_RANKS:
            raise ValueError("sweep merge supports at most %d ranks per group" % MAX_RANKS)
        if comm_dtype != "fp32":
            raise ValueError("only fp32 merge messages are supported (touch counts are exact "
                             "integers in the message buffer)")
        f = dict(dtype=torch.float32, device=self.device)
        self.start = torch.empty((self.P, 32), **f)
        self.buf = torch.empty((self.P, 16), **f)
        self.vst = torch.tensor(vst_table(), **f)
        self.comm_bytes = self.buf.numel() * 4
        self.windows = 0

    def begin(self, roster) -> None:
        self.start.copy_(roster.state)

    def messages(self, roster) -> torch.Tensor:
        native().sweep_delta(self.start, roster.state, roster.attrs, self.vst,
                             float(self.cfg.unknown_player_sigma), self.buf)
        return self.buf

    def reduce(self) -> None:
        if self.world > 1:
            dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)

    def apply(self, roster) -> None:
        native().sweep_apply(self.start, self.buf, roster.attrs, roster.state, self.vst,
                             float(self.cfg.unknown_player_sigma))
        roster.epoch = roster.epoch if roster.epoch is not None else 0  # apply wrote tag 0

    def merge(self, roster) -> None:
        """Combine every rank's window into the replicated roster (in place)."""
        if self.world <= 1:
            self.windows += 1
            return
        self.messages(roster)
        self.reduce()
        self.apply(roster)
        self.windows += 1


def rate_window_dp(rater, merger: SweepMerger, roster, rec, K=None, out=None, check=True):
    """One DP step: exact local rating of this rank's shard + posterior merge."""
    merger.begin(roster)
    res = rater.rate(roster, rec, K, out=out, check=check)
    merger.merge(roster)
    return res
