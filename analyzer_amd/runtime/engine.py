"""Streaming rating engine: window pipeline over HIP streams.

The reference processes one batch at a time, strictly serially: fetch ->
rate -> commit -> ack (/root/reference/worker.py:103-199).  Here a stream of
windows flows through two device queues:

* side stream: the schedule prepass of window i+1 (radix sort, links, deps --
  bandwidth-bound) ...
* main stream: ... runs while window i is rated by the dataflow launch
  (latency-bound), then the optional data-parallel posterior merge.

Two schedule buffer sets alternate; events order "schedule(i+1) may reuse the
set that rate(i-1) consumed" and "rate(i) needs schedule(i)".  On the CPU the
same API runs the host mirror sequentially.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Iterable, Iterator, List, Optional

import torch

from ..ops.rate import BatchRater, RateResult, Roster, Schedule
from ..utils.trace import trace_range


@dataclass
class Prepared:
    rec: torch.Tensor
    schedule: Optional[Schedule]
    ready: Optional[torch.cuda.Event]
    buffer_set: int = 0


class WindowPipeline:
    """Rate consecutive windows against one roster, prepass overlapped."""

    def __init__(self, rater: BatchRater, roster: Roster, K: int, merger=None):
        self.rater = rater
        self.roster = roster
        self.K = int(K)
        self.merger = merger
        self.device = roster.device
        self.cuda = self.device.type == "cuda"
        self.side = self._side_stream() if self.cuda else None
        self._set = 0
        self._free: List[Optional[torch.cuda.Event]] = [None, None]
        self.windows_rated = 0

    def _side_stream(self):
        """Side stream of the prepass; ``ANA_PREPASS_CUS=n`` confines it to n CUs
        (HIP CU mask) so it trickles alongside the executor instead of bursting."""
        import os

        if os.environ.get("ANA_PREPASS_SERIAL", "") not in ("", "0"):
            return torch.cuda.current_stream(self.device)  # no overlap (A/B)
        n = int(os.environ.get("ANA_PREPASS_CUS", "0") or 0)
        if n > 0:
            from ..ops.native import native

            handle = native().cu_masked_stream(self.device.index or 0, n)
            return torch.cuda.ExternalStream(handle, device=self.device)
        return torch.cuda.Stream(self.device)

    def prepare(self, rec: torch.Tensor) -> Prepared:
        """Enqueue the schedule prepass of ``rec`` on the side stream."""
        if not self.cuda:
            return Prepared(rec, None, None)
        tag = "_set%d" % self._set
        main = torch.cuda.current_stream(self.device)
        produced = torch.cuda.Event()
        produced.record(main)  # rec was produced on the main stream
        with torch.cuda.stream(self.side), trace_range("schedule", window=self.windows_rated + 1):
            self.side.wait_event(produced)
            if self._free[self._set] is not None:  # previous user of this buffer set is done
                self.side.wait_event(self._free[self._set])
            sched = self.rater.schedule(rec, self.K, self.roster.num_players, tag=tag)
            ready = torch.cuda.Event()
            ready.record(self.side)
        used = self._set
        self._set ^= 1
        return Prepared(rec, sched, ready, used)

    def rate(self, prep: Prepared, out: Optional[RateResult] = None, check: bool = False,
             telemetry=None) -> RateResult:
        """Rate a prepared window on the main stream (+ DP merge if configured);
        ``telemetry`` = (evoff, events, stats) aggregates K8 stats in the same launch."""
        main = torch.cuda.current_stream(self.device) if self.cuda else None
        if prep.ready is not None:
            main.wait_event(prep.ready)
        if self.merger is not None:
            self.merger.begin(self.roster)
        with trace_range("rate", window=self.windows_rated, matches=int(prep.rec.shape[0])):
            res = self.rater.rate(self.roster, prep.rec, self.K, out=out, check=check,
                                  schedule=prep.schedule, telemetry=telemetry)
        if self.cuda:
            done = torch.cuda.Event()
            done.record(main)
            # the buffer set of this schedule is free once this launch finished
            self._free[prep.buffer_set] = done
        if self.merger is not None:
            with trace_range("merge", window=self.windows_rated):
                self.merger.merge(self.roster)
        self.windows_rated += 1
        return res

    def run(self, windows: Iterable[torch.Tensor], out: Optional[RateResult] = None,
            on_result: Optional[Callable[[int, RateResult], None]] = None) -> int:
        """Rate every window in order; the prepass of window i+1 overlaps window i."""
        it: Iterator[torch.Tensor] = iter(windows)
        try:
            nxt = self.prepare(next(it))
        except StopIteration:
            return 0
        n = 0
        while nxt is not None:
            cur = nxt
            try:
                nxt = self.prepare(next(it))
            except StopIteration:
                nxt = None
            res = self.rate(cur, out=out)
            if on_result is not None:
                on_result(n, res)
            n += 1
        return n
