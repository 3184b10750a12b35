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

Placement (``ANA_PREPASS_SERIAL``, default auto): the prepass overlaps the executor's
tail when the executor leaves room for it, else it runs on the main stream between
launches.  Room meant 5v5 until round 6 (config 3: 22.12 ms overlapped at 0.7 vs
22.9-23.2 ms serial, profiles/r2/prepass_placement.log; since the 5v5 executor holds two
chunks, serial is faster: 19.23-19.27 vs 19.66-19.73 ms, profiles/r6/config3_held_chunks.log),
and, since round 5, a launch of one wave per SIMD
(ops/rate.py launch_blocks: 1v1-3v3 over a roster the Infinity Cache holds), whose
spare wave slots the sort fills: config 2 7.69 ms overlapped at 0.75 vs 7.95 serial,
config 4 8.62 vs 8.85 (profiles/r5/prepass_overlap_grid256.log).  At two waves per
SIMD (512 workgroups: config 5) the 1v1-3v3 launch takes a 128-VGPR build
(csrc/dataflow.hip WPE) that leaves a sort workgroup room: config 5 11.19 ms overlapped
from 0.1 vs 11.73 serial (profiles/r5/executor_vgpr_cap.log).  Without that room the
co-running prepass waits for executor workgroups to exit, or slows the executor by more
than it hides (round 2: config 2 8.07 ms serial vs 8.34-8.47 overlapped); 4v4 at 512
workgroups stays serial.
``ANA_PREPASS_CUS=n`` confines an overlapped prepass to n CUs, and with
``ANA_PREPASS_EXCLUSIVE=1`` the rating launches get the other CUs; both measured
slower than the defaults (profiles/r2/prepass_cu_mask.log, prepass_exclusive_cus.log).

Tail overlap (``ANA_PREPASS_AT``, fraction of the window, default 0.7; 0.75 at one wave
per SIMD): the
prepass of window i+1 does not start with rate(i) -- co-running the two for the
whole launch costs the latency-bound executor about as much as the prepass
itself -- but when rate(i) reaches its tail: the executor stores its launch
number to a signal-memory word once the chunks from that fraction of the window
on are being claimed, and the side stream waits on that word
(hipStreamWaitValue64).  The rest of the launch is draining in-flight
dependency chains and leaves most of the machine idle.  ``step()`` enqueues in
that order (rate(i), then prepare(i+1)); ``0`` restores start-to-start overlap.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Iterable, Iterator, List, Optional

import os

import torch

from ..config import EngineConfig
from ..ops.rate import BatchRater, RateResult, Roster, Schedule
from ..utils.trace import trace_range

CHUNK = 64  # matches per executor ticket of a window (csrc/dataflow.hip kChunk; BatchRater.chunk_len)
DP_TAIL_AT = 0.9  # tail-overlap start of the next prepass between DP merges (see tail_point)
SPARE_TAIL_AT = 0.55  # ... of a window launch at one wave per SIMD (config 2, one held chunk: 0.45-0.65
#                       6.87-6.90 ms vs 7.10 at 0.75, profiles/r6/tail_points.log; 0.75 with four held chunks)
FULL_TAIL_AT = 0.1  # ... of a 1v1-3v3 launch at two waves per SIMD (config 5: 0-0.7 swept)
WIDE_TAIL_AT = 0.5  # ... of a 5v5 launch at one wave per SIMD (config 3: 14.36-14.48 ms from 0.3-0.5,
#                     14.44-14.64 from 0.7, 14.85-15.04 from 0.85, serial 15.22-15.47,
#                     profiles/r6/wide_teams_grid_chunk.log)
DP_DEFER_AT = 0.8  # split DP merge: the deferred prefix exchange + record correction of window w
#                    start once rating w+1 claimed this fraction of its chunks (ANA_DP_DEFER_AT)


@dataclass
class Prepared:
    rec: torch.Tensor
    schedule: Optional[Schedule]
    ready: Optional[torch.cuda.Event]
    buffer_set: int = 0


class WindowPipeline:
    """Rate consecutive windows against one roster, prepass overlapped."""

    def __init__(self, rater: BatchRater, roster: Roster, K: int, merger=None, signal_at: float = 0.0,
                 telemetry: bool = False, depth: Optional[int] = None):
        self.rater = rater
        self.roster = roster
        self.K = int(K)
        self.merger = merger
        self.device = roster.device
        self.cuda = self.device.type == "cuda"
        self._set = 0
        self.windows_rated = 0
        # tail overlap: signal word + number of the last enqueued rate launch
        self.ecfg = EngineConfig.from_env()
        dp = merger is not None
        # the executor's grid for this roster (BatchRater.launch_blocks): at 256 workgroups
        # (one wave per SIMD) the overlapped prepass has wave slots of its own
        self.grid = rater.launch_blocks(self.K, roster.state.numel() * roster.state.element_size())
        self.serial = self.serial_prepass(self.K, self.ecfg, dp, self.grid)
        # DP over real collectives: the placement depends on what one merge's
        # all-reduce costs on this interconnect (probe_placement)
        self.allreduce_probe_ms: Optional[float] = None
        if dp and self.cuda and self.ecfg.prepass_serial is None and \
                (getattr(merger, "world", 1) > 1 or getattr(merger, "emulate", None) is not None):
            self.serial = self.probe_placement(merger)
        # serial prepass: nothing to overlap, no tail signal -- unless a caller wants the
        # launches' tail for other work (``signal_at``: bench.py --telemetry-mode tail),
        # which then also starts an overlapped prepass
        # (the 0.1 start of two-waves-per-SIMD 1v1-3v3 windows assumes the 128-VGPR build,
        # which launches without fused telemetry and outside the timing build only:
        # ``capped``, csrc/dataflow.hip ANA_RATE_LAUNCH_D)
        capped = not telemetry and not self.ecfg.rate_diag
        self.tail = float(signal_at) if signal_at > 0 else (
            0.0 if self.serial else self.tail_point(self.K, self.ecfg, dp, self.grid, capped))
        # a prepass in the rating's tail streams its sort input with non-temporal loads
        # (ANA_SORT_NT=2), so it evicts less of the roster the executor's drain reads:
        # eight 1.25M windows with forced merges 9.08-9.13 vs 9.32-9.40 ms (with the merge
        # kernels' non-temporal operands), config 3 20.15-20.18 vs 20.26-20.34 ms; a serial
        # prepass gains nothing (config 2: 8.00 vs 7.98; profiles/r4/merge_nt_and_sort_nt.log)
        self.sort_nt = 2 if not self.serial else -1
        # the split DP merge's deferred work (parallel/sweep.py merge_split) waits for the next
        # rating's tail: started right behind the decode it co-runs with the launch's ramp
        # and slows the rating by more than it takes (ANA_DP_DEFER_AT; <= 0: ungated)
        self.defer_at = 0.0
        if dp and self.cuda and getattr(merger, "split", None) is not None and merger.split() and \
                getattr(merger, "correct", False) and (merger.world > 1 or getattr(merger, "force", False)):
            env = os.environ.get("ANA_DP_DEFER_AT")
            self.defer_at = float(env) if env else DP_DEFER_AT
            if self.defer_at > 0 and self.tail == 0:
                self.tail = self.defer_at
        # windows prepared ahead of the one being rated (``depth``, ANA_PREPASS_DEPTH): the
        # caller prepares window i + depth behind rate(i)'s tail; depth + 1 schedule buffer
        # sets rotate.  Two lets the prepass of window i + 2 run beside the whole of rate(i+1)
        # instead of only rate(i)'s tail (overlapped placements only)
        d = depth if depth is not None else int(os.environ.get("ANA_PREPASS_DEPTH") or 0)
        self.depth = self.prepass_depth(self.K, self.grid, self.serial, dp) if d <= 0 else \
            (1 if self.serial or dp else int(d))
        self._free: List[Optional[torch.cuda.Event]] = [None] * (self.depth + 1)
        self._signal = 0
        self._seq = 0
        self.side = self._side_stream() if self.cuda else None
        # serial prepass + DP merge: the next window's prepass runs on a stream of its
        # own, beside this window's merge (messages, all-reduce, decode) -- the two
        # share nothing (the prepass reads records, the merge the roster) -- instead of
        # between the all-reduce launch and the decode on the main stream
        self.merge_side = torch.cuda.Stream(self.device) if self.cuda and self.serial else None
        self._rated: Optional[torch.cuda.Event] = None  # the last rating launch finished
        self._warm_sink: Optional[torch.Tensor] = None  # ANA_ROSTER_WARM scratch word block
        # roster warm-up before each launch: ANA_ROSTER_WARM, auto = between DP merges
        # (k short windows per step, where the rows' first reads dominate)
        self.warm = self.ecfg.roster_warm if self.ecfg.roster_warm is not None else dp
        # ANA_PREPASS_EXCLUSIVE (with ANA_PREPASS_CUS=n): the rating launches go to a
        # stream masked to the other CUs, so the two never share a CU
        self.exec_stream = None
        if self.cuda and not self.serial and self.ecfg.prepass_cus > 0 and self.ecfg.prepass_exclusive:
            from ..ops.native import native

            handle = native().cu_masked_stream(self.device.index or 0, self.ecfg.prepass_cus, True)
            self.exec_stream = torch.cuda.ExternalStream(handle, device=self.device)
        if self.cuda and self.tail > 0:
            from ..ops.native import native

            dev = self.device.index or 0
            if native().can_wait_value(dev):
                self._signal = native().progress_signal(dev)
        if self._signal and self.defer_at > 0:
            merger.defer_gate = self._gate_next

    @staticmethod
    def prepass_depth(K: int, grid: int, serial: bool, dp: bool) -> int:
        """Windows prepared ahead by default: 1 (see ``depth``)."""
        return 1

    @staticmethod
    def serial_prepass(K: int, ecfg: EngineConfig, dp: bool = False, grid: int = 512) -> bool:
        """Prepass on the main stream?  ``ANA_PREPASS_SERIAL`` if set, else serial for 4v4 and
        5v5 at two waves per SIMD (``grid`` 512: a roster past the Infinity Cache), where a
        sort workgroup does not fit beside the executor's waves -- 1v1-3v3 launches are
        compiled to leave it room (csrc/dataflow.hip ANA_EXEC_WPE); under DP merges (``dp``)
        the windows are short and the placement follows the collective's cost
        (probe_placement).  At 512 workgroups the serial prepass was faster for config 3
        (19.23-19.27 vs 19.66-19.73 ms, profiles/r6/config3_held_chunks.log); at one wave
        per SIMD (its default since the 32-match 5v5 chunks) the tail overlap is
        (14.36-14.48 vs 15.22-15.47 ms, profiles/r6/wide_teams_grid_chunk.log)."""
        if ecfg.prepass_serial is not None:
            return ecfg.prepass_serial
        return K >= 4 and not dp and grid >= 512

    def probe_placement(self, merger) -> bool:
        """Windows between DP merges: serial placement (the next prepass on its own
        stream beside the merge's collective) or the tail overlap.  Rounds 3-5 went serial
        once one merge's all-reduce cost more than 40 us (profiles/r3/
        dp_prepass_placement_k8.log: the collective exposed in the tail placement ran under
        the prepass in the serial one).  With the one-held-chunk executor (round 6) the tail
        wins at one wave per SIMD even beside an emulated N = 8 collective: config 2
        10.90-11.00 ms per step from 0.9 against 11.12-11.16 beside the merge
        (profiles/r6/tail_points.log), so there the threshold is off; at two waves per SIMD
        (512 workgroups: configs 3 and 5) serial stays faster (config 3 26.75-26.96 vs
        27.26-27.33 ms from 0.7, config 5 15.69 vs 16.06 from 0.9, profiles/r6/
        dp_placement.log).  ``ANA_DP_SERIAL_AR_US`` restores the threshold.  The probe still
        times one merge's all-reduce on this group (the max over ranks, identical
        everywhere) and reports it (``allreduce_probe_ms``)."""
        from ..parallel.comm import time_all_reduce

        if getattr(merger, "world", 1) <= 1 and getattr(merger, "emulate", None) is not None:
            ms = merger.emulated_us(int(merger.comm_bytes)) / 1000.0  # the modelled collective
        else:
            buf = torch.zeros(max(1, int(merger.comm_bytes) // 2), dtype=torch.bfloat16, device=self.device)
            ms = time_all_reduce(buf, getattr(merger, "group", None))
            del buf
        self.allreduce_probe_ms = ms
        thr = os.environ.get("ANA_DP_SERIAL_AR_US")
        if thr is not None:
            return ms > float(thr) / 1000.0
        return self.grid >= 512

    @staticmethod
    def tail_point(K: int, ecfg: EngineConfig, dp: bool = False, grid: int = 512, capped: bool = True) -> float:
        """Where the overlapped prepass starts: ``ANA_PREPASS_AT`` if set, else 0.7,
        WIDE_TAIL_AT for 5v5 windows at one wave per SIMD, DP_TAIL_AT for windows between
        merges (measured: config 2 with 8 merges
        per step, profiles/r3/dp_prepass_placement_k8.log), SPARE_TAIL_AT for 1v1-4v4
        windows at one wave per SIMD, FULL_TAIL_AT for 1v1-3v3 windows at two when the
        launch takes the 128-VGPR build (``capped``: no fused telemetry, no timing build --
        the uncapped build leaves a sort workgroup no room, so its prepass starts at 0.7)."""
        if ecfg.prepass_at_set:
            return ecfg.prepass_at
        if K >= 5 and not dp:
            return WIDE_TAIL_AT if grid < 512 else ecfg.prepass_at
        if dp:
            # (5v5 between 16 merges per step, emulated N = 8: 22.97-23.00 ms from 0.9, 23.69-23.75
            # from 0.7, 24.45 from 0.5, 23.24-23.39 beside the merge, profiles/r6/dp_placement.log)
            return DP_TAIL_AT
        if grid < 512:
            return SPARE_TAIL_AT
        return FULL_TAIL_AT if K <= 3 and capped else ecfg.prepass_at

    def _side_stream(self):
        """Side stream of the prepass; ``ANA_PREPASS_CUS=n`` confines it to n CUs
        (HIP CU mask) so it trickles alongside the executor instead of bursting."""
        if self.serial:
            return torch.cuda.current_stream(self.device)  # no overlap
        n = self.ecfg.prepass_cus
        if n > 0:
            from ..ops.native import native

            handle = native().cu_masked_stream(self.device.index or 0, n)
            return torch.cuda.ExternalStream(handle, device=self.device)
        return torch.cuda.Stream(self.device)

    def _gate_next(self, stream) -> None:
        """Make ``stream`` wait until the NEXT rating launch (not enqueued yet) reaches its
        tail -- the split DP merge's deferred work (``merger.defer_gate``)."""
        from ..ops.native import native

        native().stream_wait_value64(stream.cuda_stream, self._signal, self._seq + 1)

    def _release_gate(self) -> None:
        """Open a gate set by ``_gate_next`` now (stream-ordered on the main stream): before
        anything waits for the gated work while no further launch will release it."""
        if self.cuda and self._signal and getattr(self.merger, "defer_gate", None) is not None:
            from ..ops.native import native

            native().stream_write_value64(torch.cuda.current_stream(self.device).cuda_stream, self._signal,
                                          self._seq + 1)

    def _settle_correction(self, rows=None) -> None:
        """The split merge's deferred record correction of ``rows`` (all, with None) is
        done before the current stream goes on: release its gate, then wait."""
        m = self.merger
        if m is None or not hasattr(m, "wait_correction") or \
                (getattr(m, "_corr_done", None) is None and getattr(m, "_split_pending", None) is None):
            return
        if rows is not None and not m.correction_touches(rows):
            return
        self._release_gate()
        m.wait_correction(rows)

    def wait_tail(self, stream) -> bool:
        """Make ``stream`` wait until the last enqueued rating launch reached its tail
        (the fraction ``self.tail`` of its chunks claimed); False without a signal."""
        if not (self.cuda and self._signal and self._seq > 0):
            return False
        from ..ops.native import native

        native().stream_wait_value64(stream.cuda_stream, self._signal, self._seq)
        return True

    def _warm(self) -> None:
        """``ANA_ROSTER_WARM``: read the roster rows once on the main stream, behind the
        prepass that streamed the window's sort through the Infinity Cache, so the
        executor's first gathers of each player hit that cache (scripts/tune_rate.py
        --touch measured the effect, profiles/r4/touch_warm_roster.log; in the pipeline:
        profiles/r4/roster_warm_and_lag.log).  A window over a roster that was just
        rated in full gains nothing; the short windows between DP merges do."""
        from ..ops.native import native

        if self._warm_sink is None:
            self._warm_sink = torch.zeros(256, dtype=torch.int32, device=self.device)
        native().warm_rows(self.roster.state, self._warm_sink)

    def prepare(self, rec: torch.Tensor,
                produced: Optional[torch.cuda.Event] = None, stream=None) -> Prepared:
        """Enqueue the schedule prepass of ``rec`` on the side stream (or ``stream``),
        after the tail of the last enqueued rate launch (tail overlap) and after
        ``produced`` (default: everything enqueued on the main stream so far,
        which is where ``rec`` was made)."""
        if not self.cuda:
            return Prepared(rec, None, None)
        tag = "_set%d" % self._set
        main = torch.cuda.current_stream(self.device)
        side = self.side if stream is None else stream
        if produced is None:
            produced = torch.cuda.Event()
            produced.record(main)
        with torch.cuda.stream(side), trace_range("schedule", window=self.windows_rated + 1):
            side.wait_event(produced)
            if self._signal and self._seq > 0:
                from ..ops.native import native

                native().stream_wait_value64(side.cuda_stream, self._signal, self._seq)
            if self._free[self._set] is not None:  # previous user of this buffer set is done
                side.wait_event(self._free[self._set])
            sched = self.rater.schedule(rec, self.K, self.roster.num_players, tag=tag, sort_nt=self.sort_nt)
            ready = torch.cuda.Event()
            ready.record(side)
        used = self._set
        self._set = (self._set + 1) % len(self._free)
        return Prepared(rec, sched, ready, used)

    def rate(self, prep: Prepared, out: Optional[RateResult] = None, check: bool = False,
             telemetry=None, overlap: Optional[Callable[[], None]] = None) -> RateResult:
        """Rate a prepared window on the main stream (+ DP merge if configured);
        ``telemetry`` = (evoff, events, stats) aggregates K8 stats in the same launch.
        ``overlap``: work the merge enqueues while its all-reduces are in flight."""
        main = torch.cuda.current_stream(self.device) if self.cuda else None
        if prep.ready is not None:
            main.wait_event(prep.ready)
        if self.merger is not None:
            if hasattr(self.merger, "rec_in_use") and self.merger.rec_in_use(prep.rec):
                raise ValueError("window records reuse the memory of the previous window's records, which its "
                                 "deferred record correction has not read yet (parallel/sweep.py rec_in_use): "
                                 "give each window its own records tensor (a ring of two suffices)")
            self.merger.begin(self.roster)
            if hasattr(self.merger, "pending_rows") and self.merger.pending_rows(out):
                self.merger.flush_correction()  # a deferred record correction of these rows
            if out is not None and getattr(out, "packed", None) is not None:
                self._settle_correction(out.packed)  # ... still running on the side stream
        progress = None
        if self._signal:
            self._seq += 1
            M = int(prep.rec.shape[0])
            blocks = self.rater.launch_blocks(self.K, self.roster.state.numel() * self.roster.state.element_size())
            cl = self.rater.chunk_len(M, self.rater.tiles(telemetry, M), blocks, self.K)
            at = int(self.tail * ((M + cl - 1) // cl))
            progress = (self._signal, self._seq, at)
        if self.warm and self.cuda:
            self._warm()
        with trace_range("rate", window=self.windows_rated, matches=int(prep.rec.shape[0])):
            if self.exec_stream is not None:
                self.exec_stream.wait_stream(main)
                with torch.cuda.stream(self.exec_stream):
                    res = self.rater.rate(self.roster, prep.rec, self.K, out=out, check=check,
                                          schedule=prep.schedule, telemetry=telemetry, progress=progress)
                main.wait_stream(self.exec_stream)
            else:
                res = self.rater.rate(self.roster, prep.rec, self.K, out=out, check=check,
                                      schedule=prep.schedule, telemetry=telemetry, progress=progress)
        if self.merger is not None:
            # causal re-sweeps (parallel/sweep.py): re-rate from the prefix of the
            # earlier ranks' messages, reusing the links (only the counters reset)
            self.merger.rated()
            while self.merger.needs_resweep():
                with trace_range("resweep", window=self.windows_rated):
                    self.merger.resweep(self.roster)
                    if prep.schedule is not None:
                        prep.schedule.deps.zero_()
                    res = self.rater.rate(self.roster, prep.rec, self.K, out=res, check=check,
                                          schedule=prep.schedule)
                self.merger.rated()
        if self.cuda:
            done = torch.cuda.Event()
            done.record(main)
            # the buffer set of this schedule is free once this launch finished
            self._free[prep.buffer_set] = done
            self._rated = done
        if self.merger is not None:
            with trace_range("merge", window=self.windows_rated):
                if hasattr(self.merger, "split") and self.merger.split():
                    # the round-6 merge: the sum on the critical path, the prefix and the
                    # record correction deferred beside the next rating (parallel/sweep.py)
                    self.merger.merge_split(self.roster, prep.rec, res, overlap=overlap)
                elif getattr(self.merger, "correct", False) and res is not None and res.packed is not None and \
                        (self.merger.world > 1 or self.merger.force):
                    # the window's records corrected by the earlier ranks' evidence (parallel/sweep.py)
                    self.merger.merge_corrected(self.roster, prep.rec, res, overlap=overlap)
                else:
                    self.merger.merge(self.roster, overlap=overlap)
        elif overlap is not None:
            overlap()
        self.windows_rated += 1
        return res

    def step(self, prep: Prepared, next_rec: Optional[torch.Tensor], **rate_kwargs):
        """Rate ``prep`` and enqueue the prepass of ``next_rec`` behind its tail.
        ``next_rec`` must already be enqueued (made) on the main stream.
        Returns (result, prepared next window or None)."""
        produced = None
        if self.cuda and next_rec is not None:
            produced = torch.cuda.Event()
            produced.record(torch.cuda.current_stream(self.device))
        if self.serial and self.merger is not None and self.cuda and next_rec is not None:
            # serial prepass + DP merge: the prepass needs no roster, so it runs on its
            # own stream from the end of this window's rating on, beside the merge's
            # message kernels, all-reduces and decodes (never beside the executor)
            held: List[Prepared] = []
            res = self.rate(prep, overlap=lambda: held.append(
                self.prepare(next_rec, produced=self._rated, stream=self.merge_side)), **rate_kwargs)
            return res, held[0]
        res = self.rate(prep, **rate_kwargs)
        nxt = self.prepare(next_rec, produced=produced) if next_rec is not None else None
        return res, nxt

    def results_ready(self, res: Optional[RateResult]) -> None:
        """Make ``res``'s records final before a consumer reads them: the DP merge
        defers each window's record correction into the next merge (parallel/sweep.py
        ``defer``), so a pending one for these rows runs now (stream-ordered)."""
        if self.merger is not None and hasattr(self.merger, "pending_rows") and self.merger.pending_rows(res):
            self.merger.flush_correction()
        if res is not None and getattr(res, "packed", None) is not None:
            self._settle_correction(res.packed)

    def finish(self) -> None:
        """End of a run of windows: the last window's deferred record correction runs
        (parallel/sweep.py) and the merge decodes' clamp counter is checked (syncs;
        ``check`` raises on a decode held at the precision floor)."""
        if self.merger is not None and hasattr(self.merger, "flush_correction"):
            self.merger.flush_correction()
        self._settle_correction()
        if self.merger is not None and hasattr(self.merger, "check"):
            self.merger.check()

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
                following = next(it)
            except StopIteration:
                following = None
            res, nxt = self.step(cur, following, out=out)
            if on_result is not None:
                self.results_ready(res)
                on_result(n, res)
            n += 1
        self.finish()
        return n
