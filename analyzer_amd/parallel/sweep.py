"""Data-parallel rating with per-window posterior merge.

Each rank holds a replica of the roster (128 B/player: 1M players = 128 MB, so
replication is the right call on 288 GB devices), rates its shard of every
window exactly and in order, and then all ranks merge what they learned with
ONE dense all-reduce of natural-parameter messages (csrc/sweep.hip):

    begin(roster)   -> snapshot the window-start roster
    <rate the local shard exactly>
    merge(roster)   -> messages against a common base -> all_reduce(SUM) over
                       RCCL/xGMI -> apply (csrc/sweep_core.h)

``merge`` runs the three stages bucketed over player rows and pipelined: the
all-reduce of bucket b (asynchronous, on the collective's own stream) runs
while the main stream computes the messages of bucket b+1 and applies bucket
b-1, so on xGMI only the first bucket's message kernel and the last bucket's
apply stay exposed.  Buckets default to 64 MB of messages (ANA_MERGE_BUCKET_MB;
0 = one bucket): a 1M-player roster (64 MB) stays one all-reduce, whose ring
keeps every link at full bandwidth and whose two kernels (~40 us each) are not
worth smaller, slower messages; a 10M-player re-rate roster (640 MB) becomes ten
64-MB reduces that hide ~0.8 ms of message/apply kernels.  Every stage is
per player, so bucketing is exact.

With one rank the merge is skipped (the exact single-GPU result stands).
Backend: ``nccl`` (RCCL on ROCm) for device tensors, ``gloo`` for CPU tests.
The reference has no counterpart: horizontal scale-out there is N worker
replicas racing on MySQL rows (/root/reference/worker.py:91,174-194).
"""
from __future__ import annotations

from typing import Optional

import os

import torch
import torch.distributed as dist

from ..config import RaterConfig
from ..models.tiers import vst_table
from ..ops.native import native

MAX_RANKS = 15  # touch counts are base-16 fields in fp32 (see csrc/sweep_core.h)
COMM_DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


class SweepMerger:
    def __init__(self, num_players: int, device, cfg: Optional[RaterConfig] = None,
                 group=None, comm_dtype: str = "fp32", bucket_rows: Optional[int] = None):
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
        if bucket_rows is None:
            mb = float(os.environ.get("ANA_MERGE_BUCKET_MB", "64"))
            bucket_rows = int(mb * (1 << 20)) // (16 * 4) if mb > 0 else self.P
        self.bucket_rows = max(1, min(int(bucket_rows), max(self.P, 1)))
        self.windows = 0

    def buckets(self):
        """Row ranges [lo, hi) of the pipelined merge."""
        return [(lo, min(lo + self.bucket_rows, self.P)) for lo in range(0, self.P, self.bucket_rows)]

    def begin(self, roster) -> None:
        self.start.copy_(roster.state)

    def messages(self, roster, lo: int = 0, hi: Optional[int] = None) -> torch.Tensor:
        hi = self.P if hi is None else hi
        native().sweep_delta(self.start[lo:hi], roster.state[lo:hi], roster.attrs[lo:hi], self.vst,
                             float(self.cfg.unknown_player_sigma), self.scaled, self.buf[lo:hi])
        return self.buf

    def _launch_reduce(self, lo: int, hi: int):
        """Start the all-reduce of rows [lo, hi); returns a finisher that waits
        for it (stream-ordered, the host does not block on RCCL) and unpacks."""
        buf = self.buf[lo:hi]
        if not self.scaled:
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return work.wait
        msg = buf[:, :14].to(COMM_DTYPES[self.comm_dtype])
        touch = buf[:, 14:].to(torch.int32)
        w_msg = dist.all_reduce(msg, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        w_touch = dist.all_reduce(touch, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

        def finish():
            w_msg.wait()
            w_touch.wait()
            buf[:, :14].copy_(msg)
            buf[:, 14:].copy_(touch)
        return finish

    def reduce(self, lo: int = 0, hi: Optional[int] = None) -> None:
        if self.world <= 1:
            return
        self._launch_reduce(lo, self.P if hi is None else hi)()

    def apply(self, roster, lo: int = 0, hi: Optional[int] = None) -> None:
        hi = self.P if hi is None else hi
        native().sweep_apply(self.start[lo:hi], self.buf[lo:hi], roster.attrs[lo:hi],
                             roster.state[lo:hi], self.vst, float(self.cfg.unknown_player_sigma),
                             self.scaled)
        roster.epoch = roster.epoch if roster.epoch is not None else 0  # apply wrote tag 0

    def merge(self, roster) -> None:
        """Combine every rank's window into the replicated roster (in place):
        messages -> all-reduce -> apply, pipelined over row buckets."""
        if self.world <= 1:
            self.windows += 1
            return
        pending = None  # (lo, hi, finisher) of the bucket whose reduce is in flight
        for lo, hi in self.buckets():
            self.messages(roster, lo, hi)
            fin = self._launch_reduce(lo, hi)
            if pending is not None:
                plo, phi, pfin = pending
                pfin()
                self.apply(roster, plo, phi)
            pending = (lo, hi, fin)
        if pending is not None:
            plo, phi, pfin = pending
            pfin()
            self.apply(roster, plo, phi)
        self.windows += 1


def rate_window_dp(rater, merger: SweepMerger, roster, rec, K=None, out=None, check=True):
    """One DP step: exact local rating of this rank's shard + posterior merge."""
    merger.begin(roster)
    res = rater.rate(roster, rec, K, out=out, check=check)
    merger.merge(roster)
    return res
