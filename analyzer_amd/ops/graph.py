"""Micro-batch rating replayed as ONE HIP graph (SURVEY P3 / A2 streaming path).

The reference worker rates one batch of <= BATCHSIZE (500) matches per DB
transaction (/root/reference/worker.py:18,169-199).  On the GPU such a batch is
launch-bound: the schedule prepass (3 radix passes of upsweep / rowscan /
downsweep, the link fix-up, memsets) and the dataflow launch are ~15 small
dispatches whose issue cost is larger than their work.  ``GraphRater``
captures that whole sequence once (``torch.cuda.CUDAGraph`` = hipGraph on ROCm)
for a fixed batch capacity against a device-resident roster, and each batch is
one graph replay:

* the batch's records are copied into a static buffer; slots past the batch
  hold no-op records (unsupported mode: no state is read or written, the
  schedule keys them past the last player), so any batch size up to the
  capacity replays the same graph;
* the dataflow launch reads its tag epoch from device memory
  (``RateParams::epoch_ptr``); the graph's schedule kernel bumps it
  before every launch, so replays never see each other's granule tags.  Before
  the epoch would pass 255 the host resets the roster's tags and the counter
  (eagerly, outside the graph), exactly like ``Roster.next_epoch``;
* error flags are not read inside the graph (no host sync): ``check()`` reads
  them after a replay.

Results are bit-identical to ``BatchRater.rate`` on the same batches
(``tests/test_engine_gpu.py``).
"""
from __future__ import annotations

from typing import Optional

import torch

from .native import native
from .rate import BatchRater, RateResult, Roster

NOOP_MODE = 255  # csrc/common.h kModeUnsupported


def noop_records(n: int, K: int, device) -> torch.Tensor:
    """``[n, 2K+2]`` records that rate as 'unsupported mode' (touch nothing)."""
    rec = torch.full((n, 2 * K + 2), -1, dtype=torch.int32, device=device)
    rec[:, 2 * K] = NOOP_MODE
    rec[:, 2 * K + 1] = 0
    return rec


class EpochClock:
    """The device launch epoch of every graph that rates one roster.

    Granule tags are only unambiguous if no two launches since the last tag
    reset used the same epoch, so graphs of different team sizes (or
    capacities) over one roster must share ONE counter: each replay bumps it on
    the device, and before it would pass 255 the host resets the roster's tags
    and the counter (eagerly, outside the graphs)."""

    MAX_EPOCH = 255

    def __init__(self, roster: Roster):
        self.roster = roster
        self.epoch = torch.zeros(1, dtype=torch.int32, device=roster.device)
        self.bumps = 0
        # the graphs own the roster's tags from here on: start from a clean slate, and
        # make any later eager launch (Roster.next_epoch) reset them first
        native().reset_tags(roster.state)
        roster.epoch = None

    def before_launch(self) -> None:
        if self.bumps + 1 >= self.MAX_EPOCH:  # the next bump would reuse a live epoch
            native().reset_tags(self.roster.state)
            self.epoch.zero_()
            self.bumps = 0
            self.roster.epoch = None

    def launched(self) -> None:
        self.bumps += 1


class GraphRater:
    """Rate batches of up to ``capacity`` matches against ``roster`` by graph replay."""

    MAX_EPOCH = EpochClock.MAX_EPOCH

    def __init__(self, roster: Roster, K: int, capacity: int, rater: Optional[BatchRater] = None,
                 clock: Optional[EpochClock] = None):
        dev = roster.device
        if dev.type != "cuda":
            raise ValueError("GraphRater needs a device roster")
        self.roster, self.K, self.capacity = roster, int(K), int(capacity)
        self.rater = rater or BatchRater()
        self.rec = noop_records(self.capacity, self.K, dev)
        self.out = RateResult.allocate(self.capacity, self.K, dev)
        self.clock = clock if clock is not None else EpochClock(roster)
        self.epoch = self.clock.epoch
        self._filled = 0  # records of the last batch (the rest are no-ops)
        # warm-up outside capture (allocates the schedule workspaces), then capture
        self.clock.before_launch()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.clock.launched()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()

    @property
    def _bumps(self) -> int:
        return self.clock.bumps

    def _body(self) -> None:
        # rate() bumps the device epoch before its launch reads it (inside the schedule)
        self.rater.rate(self.roster, self.rec, self.K, out=self.out, check=False,
                        epoch_dev=self.epoch)

    def rate(self, rec: torch.Tensor) -> RateResult:
        """Rate ``rec [m, 2K+2]`` (m <= capacity, on the device) in order; the
        roster is updated in place.  Returns views of the first m result rows
        (valid until the next call)."""
        m = int(rec.shape[0])
        if m > self.capacity or rec.shape[1] != 2 * self.K + 2:
            raise ValueError("batch of shape %s does not fit capacity %d, K=%d"
                             % (tuple(rec.shape), self.capacity, self.K))
        self.rec[:m].copy_(rec)
        if m < self._filled:
            self.rec[m:self._filled].copy_(noop_records(self._filled - m, self.K, rec.device))
        self._filled = m
        self.clock.before_launch()
        self.graph.replay()
        self.clock.launched()
        o = self.out
        return RateResult(o.quality[:m], o.status[:m], o.s_mu[:m], o.s_sig[:m], o.delta[:m],
                          o.m_mu[:m], o.m_sig[:m], packed=o.packed[:m])

    def check(self) -> None:
        """Raise if the last replay set an error flag (syncs)."""
        self.rater.check_errors(self.roster.device)


__all__ = ["EpochClock", "GraphRater", "noop_records"]
