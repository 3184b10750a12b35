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
COMM_DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


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
        if comm_dtype not in COMM_DTYPES:
            raise ValueError("comm_dtype must be one of %s" % sorted(COMM_DTYPES))
        # fp16/bf16: messages use the base-relative encoding (sweep_core.h) and
        # travel compressed; the touch counters travel separately as int32
        self.comm_dtype = comm_dtype
        self.scaled = comm_dtype != "fp32"
        f = dict(dtype=torch.float32, device=self.device)
        self.start = torch.empty((self.P, 32), **f)
        self.buf = torch.empty((self.P, 16), **f)
        self.vst = torch.tensor(vst_table(), **f)
        self.comm_bytes = self.P * (16 * 4 if not self.scaled else
                                    14 * torch.finfo(COMM_DTYPES[comm_dtype]).bits // 8 + 2 * 4)
        self.windows = 0

    def begin(self, roster) -> None:
        self.start.copy_(roster.state)

    def messages(self, roster) -> torch.Tensor:
        native().sweep_delta(self.start, roster.state, roster.attrs, self.vst,
                             float(self.cfg.unknown_player_sigma), self.scaled, self.buf)
        return self.buf

    def reduce(self) -> None:
        if self.world <= 1:
            return
        if not self.scaled:
            dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)
            return
        msg = self.buf[:, :14].to(COMM_DTYPES[self.comm_dtype])
        touch = self.buf[:, 14:].to(torch.int32)
        dist.all_reduce(msg, op=dist.ReduceOp.SUM, group=self.group)
        dist.all_reduce(touch, op=dist.ReduceOp.SUM, group=self.group)
        self.buf[:, :14].copy_(msg)
        self.buf[:, 14:].copy_(touch)

    def apply(self, roster) -> None:
        native().sweep_apply(self.start, self.buf, roster.attrs, roster.state, self.vst,
                             float(self.cfg.unknown_player_sigma), self.scaled)
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
