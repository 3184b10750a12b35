"""Data-parallel rating with per-window posterior merge.

Each rank holds a replica of the roster (128 B/player: 1M players = 128 MB, so
replication is the right call on 288 GB devices), rates its shard of every
window exactly and in order, and then all ranks merge what they learned with
ONE dense all-reduce of natural-parameter messages (csrc/sweep.hip):

    begin(roster)   -> the common window start (kept by the last merge: no copy)
    <rate the local shard exactly>
    merge(roster)   -> messages against the start -> all_reduce(SUM) over
                       RCCL/xGMI -> decode into the roster AND the next start

``merge`` runs the three stages bucketed over player rows and pipelined: the
all-reduce of bucket b (asynchronous, on the collective's own stream) runs
while the main stream computes the messages of bucket b+1 and decodes bucket
b-1, so on xGMI only the first bucket's message kernel and the last bucket's
decode stay exposed.  Buckets default to 64 MB of messages (ANA_MERGE_BUCKET_MB;
0 = one bucket): the 1M-player operands (32 B per player with fp16 / bf16
messages) stay one all-reduce, a 10M-player re-rate roster (320 MB) becomes five,
each big enough to run the xGMI links at bandwidth, so the message kernel of
bucket b+1 and the decode of bucket b-1 hide behind the collective.  Emulated
N = 2 (profiles/r6/dp_bucketed_merge.log): config 5 13.02-13.04 ms per step at
64 MB, 13.14-13.16 at 16 MB, 13.44-13.45 whole; config 2 7.57-7.60 either way.
Every stage is per player, so bucketing is exact.

**Causal re-sweeps (``sweeps`` > 1).**  Rank r's shard is the r-th time slice
of the global window (bench.py, runtime/rerate.py), so under the reference's
exact semantics (ORDER BY created_at + a sequential loop,
/root/reference/worker.py:176,191-192) rank r's matches must see the
posteriors of ranks 0..r-1.  One sweep rates every shard from the window start
(the approximation).  A re-sweep re-rates shard r from

    prior_r = start + sum_{q<r} message_q      (exclusive prefix over ranks,
                                                 comm.exclusive_scan)

and measures the new message from that prior (sweep_core.h), so the prefix
telescopes: after sweep s, ranks 0..s-1 hold their exact posteriors, and
``sweeps == world`` reproduces the sequential result up to fp32 rounding of the
natural-parameter round trip.  ``parallel/accuracy.py`` measures the error per
sweep count.  This is deliberately a prefix, not the EP cavity (merged / own
message): the cavity would feed later ranks' evidence into earlier matches,
which converges to a smoother, not to the reference's filter.

**Causal record correction (``correct_records``, default on for one sweep).**  Rank
r's records miss the evidence of the earlier slices (ranks q < r) that the
reference's sequential loop had folded in.  The merge's collective then also
returns each rank's exclusive prefix of the messages (comm.scan_and_sum: one
exchange, 1.5x an all-reduce's volume), and one pass over the window's records adds
that prefix in natural parameters before the decode (csrc/sweep_core.h
``correct_record_slot``): 8 ranks at the k = 8 density, records median |d mu| 29.7
-> 8.0 against exact sequential rating, the level of the merged roster itself
(profiles/r5/record_correction.log).

**No one-window-late merge.**  Rounds 4-5 built and removed a lagged merge (window
b's all-reduce under window b+1's rating): a message measured against the rank's
own start -- which lacks the other ranks' previous window, tau^2 dynamics included
-- overshoots the common roster's precision, and the summed messages crossed zero
in every precision (profiles/r5/lag_bf16_root_cause.log).  Every decode now counts
the tracks it had to clamp (``clamps``, ``check``).

With one rank the merge is skipped (the exact single-GPU result stands).
Backend: ``nccl`` (RCCL on ROCm) for device tensors, ``gloo`` for CPU tests.
The reference has no counterpart: horizontal scale-out there is N worker
replicas racing on MySQL rows (/root/reference/worker.py:91,174-194).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..config import EngineConfig, RaterConfig
from ..models.tiers import vst_table
from ..ops.native import native
from .comm import SplitExchange, all_reduce_sum, exclusive_scan, scan_and_sum, scan_and_sum_start, world

MAX_RANKS = 15  # touch counts are base-16 fields in fp32 (see csrc/sweep_core.h)


class MergeClampError(FloatingPointError):
    """A decode's merged precision came out at or below zero (sweep_core.h
    sweep_apply_track) and was held at the floor: the reference raises on numeric
    trouble and dead-letters the batch (/root/reference/rater.py:7-8,
    worker.py:108-120); a silently clamped sigma must never be written."""
BASE_FLOATS = 16  # base row: (mu, sigma) per 16-B granule of a roster row


def base_rows(state: torch.Tensor) -> torch.Tensor:
    """Roster rows [P, 32] -> base rows [P, 16]: (mu, sigma) of each granule."""
    return state.view(state.shape[0], 8, 4)[:, :, 0::2].reshape(state.shape[0], BASE_FLOATS)
COMM_DTYPES = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


class SweepMerger:
    def __init__(self, num_players: int, device, cfg: Optional[RaterConfig] = None,
                 group=None, comm_dtype: str = "fp32", bucket_rows: Optional[int] = None,
                 sweeps: int = 1, world_size: Optional[int] = None, force: bool = False,
                 emulate: Optional[str] = None, correct_records: Optional[bool] = None):
        self.P = int(num_players)
        self.device = torch.device(device)
        self.cfg = cfg or RaterConfig.from_env()
        self.group = group
        self.world = int(world_size) if world_size is not None else world(group)[1]
        if self.world > MAX_RANKS:
            raise ValueError("sweep merge supports at most %d ranks per group" % MAX_RANKS)
        if comm_dtype not in COMM_DTYPES:
            raise ValueError("comm_dtype must be one of %s" % sorted(COMM_DTYPES))
        self.sweeps = max(1, int(sweeps))
        # force: run the merge kernels even on one rank (the all-reduce of one rank
        # is the identity) -- bench.py --force-merge prices the merge without comm
        self.force = bool(force)
        # causal record correction (module docstring): one sweep only -- causal re-sweeps
        # already rate every slice from its exact prefix
        if correct_records is None:
            correct_records = os.environ.get("ANA_DP_CORRECT_RECORDS", "1") not in ("", "0", "false")
        self.correct = bool(correct_records) and self.sweeps <= 1
        self._zero_prefix = None  # one rank: its prefix is zero (the pass still runs: it is priced)
        # the correction of window w's records runs in merge w+1, while window w+1's
        # collective is in flight (its only input, the increment table, is ready once
        # decode w ran): ANA_DP_CORRECT_DEFER=0 runs it in line after decode w.  A rating
        # into the rows it still has to correct, finish() and results_ready() run it first
        self.defer = os.environ.get("ANA_DP_CORRECT_DEFER", "1") not in ("", "0", "false")
        self._pending = None      # (rec, K, rows, delta) of the deferred correction
        self._coll = None         # side stream of the merge's collectives (RCCL)
        self.delta = None         # [P, 16] fp32 increments of the record correction (decode_packed)
        # emulate = "N:GBps[:us]" (one rank, force): every all-reduce is replaced by a stand-in
        # on a stream of its own that takes what an N-rank ring all-reduce of the operands would
        # over links of GBps bus bandwidth (+ us latency) and streams the buffer three times on
        # 32 CUs, as RCCL's channels do (csrc/kernels.hip emulate_allreduce_kernel) -- one GPU
        # then prices the
        # N-GPU step, the merge's exposed collective included (bench.py --emulate-allreduce)
        self.emulate = None
        if emulate:
            parts = [float(x) for x in str(emulate).split(":")]
            ranks, bw = int(parts[0]), parts[1]
            lat = parts[2] if len(parts) > 2 else 25.0
            if ranks < 2 or bw <= 0:
                raise ValueError("emulate must be N:GBps[:latency_us] with N >= 2")
            self.emulate = (ranks, bw, lat)
        self._comm = None  # stream of the emulated collective
        # fp16/bf16: messages use the base-relative encoding (sweep_core.h) and
        # travel compressed; the touch counters travel separately as int32
        self.comm_dtype = comm_dtype
        self.scaled = comm_dtype != "fp32"
        f = dict(dtype=torch.float32, device=self.device)
        # common window start as BASE rows: (mu, sigma) of the 8 granules, 64 B per
        # player (csrc/sweep_core.h) -- a message needs nothing else of the row
        self.start = torch.empty((self.P, BASE_FLOATS), **f)
        self.prior = None                            # this rank's prior (re-sweeps only; base rows)
        self.buf = torch.empty((self.P, 16), **f)
        # fp16/bf16: merge() writes and reads the all-reduce operands directly
        # (messages [P, 14] in the comm dtype + the two touch-count fields packed in one
        # int32, lo | hi << 16: 32 B per player on the wire)
        self.msg = torch.empty((self.P, 14), dtype=COMM_DTYPES[comm_dtype], device=self.device) \
            if comm_dtype != "fp32" else None
        self.cnt = torch.empty((self.P, 1), dtype=torch.int32, device=self.device) \
            if comm_dtype != "fp32" else None
        # the split merge's operand rows (merge_split): [P, 16] halves = 8 words per player,
        # messages in words 0..6 and the touch word last (32 B per player on the wire), and
        # two window starts -- decode w reads one and writes the other, so window w's start
        # stays intact for its deferred record correction while window w+1 is rated
        self.op = torch.empty((self.P, 16), dtype=COMM_DTYPES[comm_dtype], device=self.device) \
            if comm_dtype != "fp32" else None
        self._starts = [self.start, None]
        # default off: on one GPU with the emulated collective the split merge measured slower
        # for config 2 at N = 8 (11.58-11.76 vs 11.22-11.26 ms per step, profiles/r6/
        # dp_split_merge.log) -- the merge slot is bandwidth-bound by the next window's prepass
        # and the record correction, not by the collective; ANA_DP_SPLIT=1 turns it on
        self.use_split = os.environ.get("ANA_DP_SPLIT", "0") not in ("", "0", "false")
        # where the deferred prefix exchange + record correction start: a callable that makes
        # a stream wait for the NEXT rating launch's tail (runtime/engine.py sets it when the
        # launches carry a tail signal, ANA_DP_DEFER_AT); None: right behind the decode
        self.defer_gate: Optional[Callable] = None
        self._side = None         # stream of the deferred record correction (merge_split)
        self._corr_done = None    # event: the last deferred correction finished
        self._pd_done = None      # event: its delta table is written (the start it read is free)
        self._split_pending = None  # the correction waiting for the next merge (defer_mode "next")
        # the corrected merge (merge_corrected) pipelined over the row buckets (messages of
        # bucket b+1 and the decode of bucket b-1 beside bucket b's collective):
        # ANA_DP_CORR_BUCKETS=1.  Off by default: emulated N = 8, config 2, 11.09 ms per step
        # with 16-MB buckets and 11.58 with 8-MB ones against 10.83-10.86 whole; config 5
        # 15.91-15.94 vs 15.67 (profiles/r6/dp_bucketed_merge.log) -- the overlapped
        # kernels slow the collective's stand-in and each other by more than they hide
        self.corr_buckets = os.environ.get("ANA_DP_CORR_BUCKETS", "0") not in ("", "0", "false")
        # ANA_DP_DEFER: "next" (default) -- window w's correction runs beside window w+1's
        # collective; "tail" -- behind the decode, gated on the next rating's tail; "now" --
        # behind the decode at once
        self.defer_mode = os.environ.get("ANA_DP_DEFER") or "next"
        self._corr_rows = None    # RateResult rows it writes
        self._corr_events: List[tuple] = []  # (begin, end) timing events on the side stream
        self.vst = torch.tensor(vst_table(), **f)
        self._none = torch.empty(0, **f)
        # decoded tracks whose merged precision hit the floor, summed over every decode
        # since the last check (sticky, on the device: no sync per merge) -- check() raises
        self.clamps = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.comm_bytes = self.P * (16 * 4 if not self.scaled else
                                    14 * torch.finfo(COMM_DTYPES[comm_dtype]).bits // 8 + 4)
        if bucket_rows is None:  # ANA_MERGE_BUCKET_MB of all-reduce operands per bucket
            mb = EngineConfig.from_env().merge_bucket_mb
            row_bytes = 16 * 4 if not self.scaled else 14 * torch.finfo(COMM_DTYPES[comm_dtype]).bits // 8 + 4
            bucket_rows = int(mb * (1 << 20)) // row_bytes if mb > 0 else self.P
        if self.world <= 1 and self.emulate is None:
            # one rank (force): no collective to overlap, so one bucket -- two launches
            # per merge instead of two per bucket (the emulated collective is bucketed like
            # the real one)
            bucket_rows = self.P
        self.bucket_rows = max(1, min(int(bucket_rows), max(self.P, 1)))
        self.windows = 0
        self._synced = False   # start == the roster as the last merge left it
        self._sweep = 0        # sweeps rated in the current window
        self.timing = False    # record per-stage CUDA events (profile())
        self._events: List[tuple] = []

    # ----------------------------------------------------------- stages
    def buckets(self):
        """Row ranges [lo, hi) of the pipelined merge."""
        return [(lo, min(lo + self.bucket_rows, self.P)) for lo in range(0, self.P, self.bucket_rows)]

    def begin(self, roster) -> None:
        """Start a window.  The common start is the roster the last merge wrote
        (the merge decodes into both), so only the first window -- or one after
        ``invalidate()`` -- copies it."""
        if not self._synced:
            self.start.copy_(base_rows(roster.state))
            self._synced = True
        self._sweep = 0

    def invalidate(self) -> None:
        """The roster was changed outside the merger: re-snapshot at the next begin."""
        self._synced = False

    def messages(self, roster, lo: int = 0, hi: Optional[int] = None) -> torch.Tensor:
        """Messages of rows [lo, hi): posterior (roster) against this sweep's prior."""
        hi = self.P if hi is None else hi
        prior = self.start if self._sweep <= 1 or self.prior is None else self.prior
        native().sweep_delta(self.start[lo:hi], prior[lo:hi], roster.state[lo:hi], roster.attrs[lo:hi],
                             self.vst, float(self.cfg.unknown_player_sigma), self.scaled, self.buf[lo:hi])
        return self.buf

    def decode(self, roster, lo: int = 0, hi: Optional[int] = None, into=None) -> None:
        """roster.state[lo:hi] (and ``into``[lo:hi]) := start + summed messages in buf."""
        hi = self.P if hi is None else hi
        s2 = into[lo:hi] if into is not None else self._none
        if self.sweeps > 1:
            # causal re-sweeps: the messages telescope (each measured from its rank's exact
            # causal prior), so their natural-parameter sum is exact -- every touch field
            # held at <= 1 keeps the decode off the variance-space branch for net losses
            # (sweep_core.h merged_ratio), which is for independent slices only
            t = self.buf[lo:hi, 14:16]
            x = t.to(torch.int32)
            t.copy_(((x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x11111111).to(t.dtype))
        native().sweep_apply(self.start[lo:hi], self.buf[lo:hi], roster.attrs[lo:hi],
                             roster.state[lo:hi], s2, self.vst, float(self.cfg.unknown_player_sigma),
                             self.scaled, self.clamps)
        roster.epoch = roster.epoch if roster.epoch is not None else 0  # decode wrote tag 0

    def messages_packed(self, roster, lo: int = 0, hi: Optional[int] = None, into=None) -> None:
        """``messages`` straight into the compressed all-reduce operands (first sweep);
        ``into`` = (msg, cnt) views (merge_split's operand rows), else ``msg`` / ``cnt``."""
        hi = self.P if hi is None else hi
        msg, cnt = into if into is not None else (self.msg, self.cnt)
        native().sweep_delta_packed(self.start[lo:hi], self.start[lo:hi], roster.state[lo:hi],
                                    roster.attrs[lo:hi], self.vst, float(self.cfg.unknown_player_sigma),
                                    msg[lo:hi], cnt[lo:hi])

    def decode_packed(self, roster, lo: int = 0, hi: Optional[int] = None, into=None,
                      prefix: Optional[torch.Tensor] = None, delta: Optional[torch.Tensor] = None) -> None:
        """``decode`` of the compressed summed messages; with ``prefix`` (this rank's
        exclusive prefix, same layout as ``msg``) it also writes the record
        correction's ``delta`` table from the window start before overwriting it."""
        hi = self.P if hi is None else hi
        s2 = into[lo:hi] if into is not None else self._none
        native().sweep_apply_packed(self.start[lo:hi], self.msg[lo:hi], self.cnt[lo:hi], roster.attrs[lo:hi],
                                    roster.state[lo:hi], s2, self.vst, float(self.cfg.unknown_player_sigma),
                                    self.clamps, None if prefix is None else prefix[lo:hi],
                                    None if delta is None else delta[lo:hi])
        roster.epoch = roster.epoch if roster.epoch is not None else 0

    def _packed(self) -> bool:
        return self.msg is not None and (self._sweep <= 1 or self.prior is None)

    # --------------------------------------------------- the split merge (round 6)
    def op_views(self):
        """(msg [P, 14], cnt [P, 1] int32) views of the split merge's operand rows."""
        return self.op[:, :14], self.op.view(torch.int32)[:, 7:8]

    def split(self) -> bool:
        """Merges of this merger go through ``merge_split`` (compressed messages, one sweep;
        ``ANA_DP_SPLIT=0``: the round-5 merges, kept as the reference the tests compare with)."""
        return self.op is not None and self.sweeps <= 1 and self.use_split

    def _emulated(self, t: torch.Tensor, nbytes: float, passes: int, stream) -> None:
        """The collective stand-in (``emulate``) over ``t`` on ``stream``: the modelled time
        of ``nbytes`` per rank over the emulated links plus one latency."""
        n, bw, lat = self.emulate
        with torch.cuda.stream(stream):
            native().emulate_allreduce(t, 32, passes, lat + nbytes / (bw * 1e3))

    def merge_split(self, roster, rec: Optional[torch.Tensor] = None, out=None,
                    overlap: Optional[Callable[[], None]] = None) -> None:
        """One window's merge with the collective split at what the next window needs
        (comm.SplitExchange): messages -> all-to-all / owner reduce / all-gather of the
        SUM -> decode into the roster and the other window start -> the next rating may
        start.  With the causal record correction (``correct`` and ``rec``/``out``) the
        prefix return (an all-to-all on the collective stream) and the correction (the
        delta table from this window's start + the prefix, then the records pass, on a
        side stream) are enqueued behind it and run beside the next window's rating.

        Round 5 ran the scan (3 (N-1)/N of the buffer) and the previous window's
        correction in front of the decode (emulated N = 8: 11.24 ms per step,
        docs/DP_PROJECTION.md)."""
        if self.world <= 1 and not self.force:
            self.windows += 1
            if overlap is not None:
                overlap()
            return
        correct = self.correct and rec is not None and out is not None and out.packed is not None
        K = (int(rec.shape[1]) - 2) // 2 if rec is not None else 0
        cuda = self.device.type == "cuda"
        main = torch.cuda.current_stream(self.device) if cuda else None
        msg, cnt = self.op_views()
        self._ev("begin")
        nxt = self._starts[1]
        if nxt is None:
            nxt = self._starts[1] = torch.empty_like(self.start)
        self.messages_packed(roster, into=(msg, cnt))
        self._ev("messages")
        words = self.op.view(torch.int32)
        n_emul = self.emulate[0] if (self.emulate is not None and self.world <= 1 and cuda) else 0
        # the previous window's record correction goes beside this merge's collective: enqueued
        # first on the side stream, it starts behind these messages (defer_mode "next")
        pending_prev = self._split_pending is not None
        if cuda and self._coll is None:
            self._coll = torch.cuda.Stream(self.device)
        prefix = None
        if self.world > 1:
            ex = SplitExchange(words, self.op.dtype, group=self.group, stream=self._coll,
                               want_prefix=correct, force=world(self.group)[1] < self.world)
            if pending_prev:
                self._enqueue_split_correction()
            if overlap is not None:
                overlap()
            self._ev("overlap")
            total = ex.total()
            get_prefix = ex.prefix
            send_prefix = (lambda: ex.send_prefix(self.defer_gate))  # noqa: E731
        else:
            # one rank (force): the sum is the operand itself and the prefix zero; with
            # ``emulate`` the stand-ins price the N-rank exchange on the collective stream --
            # the critical part (2 (N-1)/N of the buffer + the owner reduce of N blocks) in
            # front of the decode, the prefix return behind it beside the next rating
            total = words
            zero = self._prefix_zero(self.op[:, :14]).view(torch.int32) if correct else None
            get_prefix = (lambda: zero)  # noqa: E731
            send_prefix = None
            if n_emul:
                self._coll.wait_stream(main)
                nb = float(self.P * 32)
                self._emulated(words, 2.0 * (n_emul - 1) / n_emul * nb, 3, self._coll)
                blk = self.P // n_emul
                if blk > 0:
                    if getattr(self, "_emul_scratch", None) is None:
                        self._emul_scratch = (torch.empty((blk, 8), dtype=torch.int32, device=self.device),
                                              torch.empty((n_emul * blk, 7), dtype=torch.int32,
                                                          device=self.device))
                    tot_s, pref_s = self._emul_scratch
                    with torch.cuda.stream(self._coll):
                        native().sweep_block_reduce(words[:n_emul * blk], n_emul, self.op.dtype == torch.bfloat16,
                                                    tot_s, pref_s if correct else None)
                done = torch.cuda.Event()
                done.record(self._coll)
                if correct and blk > 0:  # the deferred prefix return, sent behind the decode
                    pref_ev = {}

                    def send_prefix():
                        with torch.cuda.stream(self._coll):
                            if self.defer_gate is not None:
                                self.defer_gate(self._coll)
                        self._emulated(self._emul_scratch[1], (n_emul - 1) / n_emul * self.P * 28.0, 2,
                                       self._coll)
                        pref_ev["ev"] = torch.cuda.Event()
                        pref_ev["ev"].record(self._coll)

                    get_prefix = (lambda: (torch.cuda.current_stream(self.device).wait_event(pref_ev["ev"]),  # noqa: E731
                                           zero)[1])
                if pending_prev:
                    self._enqueue_split_correction()
                if overlap is not None:
                    overlap()
                self._ev("overlap")
                main.wait_event(done)
            else:
                if pending_prev:
                    self._enqueue_split_correction()
                if overlap is not None:
                    overlap()
                self._ev("overlap")
        self._ev("allreduce")
        if cuda and self._pd_done is not None:
            # the previous window's deferred delta table read the start this decode writes
            main.wait_event(self._pd_done)
        tmsg = total.view(self.op.dtype)[:, :14] if total is not words else msg
        tcnt = total[:, 7:8] if total is not words else cnt
        native().sweep_apply_packed(self.start, tmsg, tcnt, roster.attrs, roster.state, nxt, self.vst,
                                    float(self.cfg.unknown_player_sigma), self.clamps, None, None)
        roster.epoch = roster.epoch if roster.epoch is not None else 0
        self._ev("apply")
        cur = self.start
        if correct and send_prefix is not None:
            send_prefix()  # the prefix return: gated on the next rating's tail (defer_gate)
        if correct:
            pend = dict(cur=cur, rec=rec, K=K, rows=out.packed, get_prefix=get_prefix, attrs=roster.attrs)
            self._corr_rows = out.packed
            if self.defer_mode == "next" and cuda:
                self._split_pending = pend  # beside the next merge's collective (or a flush)
            else:
                self._split_pending = pend
                self._enqueue_split_correction(gate=self.defer_gate if self.defer_mode == "tail" else None)
        self._starts = [nxt, cur]
        self.start = nxt
        self._synced = True
        self.windows += 1

    def _enqueue_split_correction(self, gate=None) -> None:
        """Enqueue the pending record correction of the split merge (``merge_split``): on
        the side stream behind everything the current stream enqueued so far (in the default
        placement: the next window's messages, so it runs beside that merge's collective,
        where the GPU is otherwise idle), the delta table from that window's start + the
        prefix, then the records pass.  Host tensors: at once."""
        pend = self._split_pending
        if pend is None:
            return
        self._split_pending = None
        cuda = self.device.type == "cuda"
        if self.delta is None:
            self.delta = torch.empty((self.P, 16), dtype=torch.float32, device=self.device)
        if cuda:
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            self._side.wait_stream(torch.cuda.current_stream(self.device))
            ctx = torch.cuda.stream(self._side)
        else:
            ctx = _NullCtx()
        with ctx:
            b = None
            if cuda and gate is not None:
                gate(self._side)
            if cuda and self.timing:
                b = torch.cuda.Event(enable_timing=True)
                b.record()
            pw = pend["get_prefix"]()
            native().prefix_delta(pend["cur"], pw.view(self.op.dtype), pend["attrs"], self.vst,
                                  float(self.cfg.unknown_player_sigma), self.delta)
            if cuda:
                self._pd_done = torch.cuda.Event()
                self._pd_done.record()
            native().correct_records(pend["rec"], pend["K"], pend["rows"], self.delta)
            if cuda:
                if b is not None:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record()
                    self._corr_events.append((b, e))
                self._corr_done = torch.cuda.Event()
                self._corr_done.record()
                for t in (pend["cur"], pend["rec"], pend["rows"], pw):
                    t.record_stream(self._side)

    def rec_in_use(self, rec) -> bool:
        """Whether a deferred record correction still has to read match records in the
        memory of ``rec`` (round-5 ``_pending`` or a pending split correction).  The records
        of window i must stay unchanged until the merge of window i+1 has been enqueued:
        a caller refilling window i's tensor in place for window i+1 would have the
        correction read the wrong player ids -- runtime/engine.py refuses such a window."""
        pend = []
        if self._pending is not None:
            pend.append(self._pending[0])
        if self._split_pending is not None:
            pend.append(self._split_pending["rec"])
        for a in pend:
            a0, b0 = a.data_ptr(), rec.data_ptr()
            if a0 < b0 + rec.numel() * rec.element_size() and b0 < a0 + a.numel() * a.element_size():
                return True
        return False

    def flush_split(self) -> None:
        """Enqueue a correction still waiting for the next merge (finish, a consumer)."""
        if self._split_pending is not None:
            self._enqueue_split_correction()

    def correction_touches(self, rows) -> bool:
        """Whether the last deferred record correction writes (part of) ``rows``."""
        if self._corr_rows is None:
            return False
        a, b = self._corr_rows, rows
        a0, b0 = a.data_ptr(), b.data_ptr()
        return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()

    def wait_correction(self, rows=None) -> None:
        """Make the current stream wait for the deferred record correction (of ``rows``,
        when given: only if it writes them); a pending one is enqueued first."""
        if rows is not None and not self.correction_touches(rows):
            return
        self.flush_split()
        if self._corr_done is None or self.device.type != "cuda":
            return
        if rows is not None and self._corr_rows is not None:
            a, b = self._corr_rows, rows
            a0, b0 = a.data_ptr(), b.data_ptr()
            if not (a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()):
                return
        torch.cuda.current_stream(self.device).wait_event(self._corr_done)

    def correction_ms(self) -> float:
        """Side-stream time of the deferred corrections since the last call (syncs)."""
        if not self._corr_events:
            return 0.0
        torch.cuda.synchronize(self.device)
        ms = sum(b.elapsed_time(e) for b, e in self._corr_events)
        self._corr_events.clear()
        return ms

    # legacy name: decode the all-reduced messages into the roster only
    def apply(self, roster, lo: int = 0, hi: Optional[int] = None) -> None:
        self.decode(roster, lo, hi)

    def rated(self) -> None:
        """The local shard was rated once more (the engine calls this after each sweep)."""
        self._sweep += 1

    # ------------------------------------------------------ collectives
    def _split(self, buf):
        if not self.scaled:
            return [buf]
        return [buf[:, :14].to(COMM_DTYPES[self.comm_dtype]), buf[:, 14:].to(torch.int32)]

    def _join(self, buf, parts) -> None:
        if self.scaled:
            buf[:, :14].copy_(parts[0])
            buf[:, 14:].copy_(parts[1])

    def _launch_reduce(self, lo: int, hi: int, packed: bool = False):
        """Start the all-reduce of rows [lo, hi); returns a finisher that waits
        for it (stream-ordered, the host does not block on RCCL) and unpacks."""
        buf = self.buf[lo:hi]
        parts = [self.msg[lo:hi], self.cnt[lo:hi]] if packed else self._split(buf)
        # one rank (force): the sum over ranks is the message itself
        works = [all_reduce_sum(t, group=self.group, async_op=True) for t in parts] if self.world > 1 else []
        if self.world <= 1 and self.emulate is not None and self.device.type == "cuda":
            return self._emulated_reduce(parts, buf, packed)

        def finish():
            for w in works:
                if w is not None:
                    w.wait()
            if not packed:
                self._join(buf, parts)
        return finish

    def emulated_us(self, nbytes: int) -> float:
        """Modelled time of an N-rank ring all-reduce of nbytes (``emulate``)."""
        n, bw, lat = self.emulate
        return lat + 2.0 * (n - 1) / n * nbytes / (bw * 1e3)

    def _emulated_reduce(self, parts, buf, packed):
        """The all-reduce stand-in (``emulate``), on its own stream after the
        messages, as RCCL runs its kernels; the finisher makes the main stream wait."""
        main = torch.cuda.current_stream(self.device)
        if self._comm is None:
            self._comm = torch.cuda.Stream(self.device)
        self._comm.wait_stream(main)
        nbytes = sum(t.numel() * t.element_size() for t in parts)
        with torch.cuda.stream(self._comm):
            for i, t in enumerate(parts):  # the time is modelled on the whole operand set
                native().emulate_allreduce(t, 32, 3, self.emulated_us(nbytes) if i == 0 else 0.0)
        done = torch.cuda.Event()
        done.record(self._comm)

        def finish():
            main.wait_event(done)
            if not packed:
                self._join(buf, parts)
        return finish

    def reduce(self, lo: int = 0, hi: Optional[int] = None) -> None:
        if self.world <= 1:
            return
        self._launch_reduce(lo, self.P if hi is None else hi)()

    def scan(self) -> None:
        """buf := sum of the messages of the ranks before this one (exclusive prefix)."""
        parts = [exclusive_scan(t, group=self.group) for t in self._split(self.buf)]
        if self.scaled:
            self._join(self.buf, parts)
        else:
            self.buf.copy_(parts[0])

    # ------------------------------------------------------------ drivers
    def needs_resweep(self) -> bool:
        return self.world > 1 and self._sweep < self.sweeps

    def resweep(self, roster) -> None:
        """Between sweeps: roster := this rank's causal prior (start + messages of
        the earlier ranks), kept in ``prior`` to measure the next message from."""
        if self.prior is None:
            self.prior = torch.empty_like(self.start)
        self.messages(roster)
        self.scan()
        self.decode(roster, into=self.prior)

    def _ev(self, name):
        if self.timing and self.device.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append((name, e))

    def _prefix_zero(self, like: torch.Tensor) -> torch.Tensor:
        if self._zero_prefix is None or self._zero_prefix.dtype != like.dtype:
            self._zero_prefix = torch.zeros_like(like)
        return self._zero_prefix

    def merge_corrected(self, roster, rec: torch.Tensor, out, overlap: Optional[Callable[[], None]] = None) -> None:
        """``merge`` with the causal record correction of this window's records
        (``rec``, RateResult ``out``): messages -> ONE collective giving the sum and
        this rank's exclusive prefix (comm.scan_and_sum) -> the decode, which also turns
        the prefix into the increment table -> the records pass.  The records name any
        player, so the pass needs the whole table; the messages, the collective and the
        decode are row-wise and pipeline over the row buckets (``corr_buckets``): bucket
        b+1's messages and bucket b-1's decode run beside bucket b's collective.

        Deferred (``defer``, default): the records pass of this window is enqueued by
        the NEXT merge right after its collectives are launched, so it runs while they
        are in flight (RCCL on its own stream; the emulated stand-in on 32 CUs)
        instead of on the critical path; ``flush_correction`` runs a pending pass."""
        K = (int(rec.shape[1]) - 2) // 2
        self._ev("begin")
        packed = self.msg is not None
        buckets = self.buckets() if (packed and self.corr_buckets) else [(0, self.P)]
        launched = []
        for lo, hi in buckets:
            if packed:
                self.messages_packed(roster, lo, hi)
            else:
                self.messages(roster)
            launched.append((lo, hi, self._launch_scan(lo, hi, packed)))
        self._ev("messages")
        self.flush_correction()  # the previous window's records, beside the collectives
        self._ev("correct")
        if overlap is not None:
            overlap()
        self._ev("overlap")
        if packed and self.delta is None:
            self.delta = torch.empty((self.P, 16), dtype=torch.float32, device=self.device)
        delta = self.delta
        for lo, hi, fin in launched:
            prefix, total = fin()
            self._ev("allreduce")
            if packed:  # the decode also turns the scaled prefix into raw increments
                if total is not self.msg[lo:hi] and total.data_ptr() != self.msg[lo:hi].data_ptr():
                    self.msg[lo:hi].copy_(total)
                native().sweep_apply_packed(self.start[lo:hi], self.msg[lo:hi], self.cnt[lo:hi],
                                            roster.attrs[lo:hi], roster.state[lo:hi], self.start[lo:hi],
                                            self.vst, float(self.cfg.unknown_player_sigma), self.clamps,
                                            prefix, delta[lo:hi])
                roster.epoch = roster.epoch if roster.epoch is not None else 0
            else:                 # raw fp32 messages: the prefix IS the increment table
                if total is not self.buf:
                    self.buf.copy_(total)
                self.decode(roster, into=self.start)
                delta = prefix
            self._ev("apply")
        self._pending = (rec, K, out.packed, delta)
        if not self.defer:
            self.flush_correction()
            self._ev("correct")
        self._synced = True
        self.windows += 1

    def _launch_scan(self, lo: int, hi: int, packed: bool):
        """Start the scan-and-sum collective of rows [lo, hi) (comm.scan_and_sum_start on
        the collective stream); returns ``finish() -> (prefix, total)`` of those rows.  One
        rank (force): the prefix is zero and the total the operand -- with ``emulate`` the
        stand-in prices the N-rank exchange, 1.5x an all-reduce's volume."""
        operand = self.msg[lo:hi] if packed else self.buf
        if self.world > 1:
            if self._coll is None and self.device.type == "cuda":
                self._coll = torch.cuda.Stream(self.device)
            # (force: a world_size override above the group's real size runs the exchanges
            # anyway -- the one-rank RCCL test of this path)
            return scan_and_sum_start(operand, group=self.group, stream=self._coll,
                                      extra=self.cnt[lo:hi] if packed else None,
                                      force=world(self.group)[1] < self.world)
        prefix0 = self._prefix_zero(self.msg)[lo:hi] if packed else self._prefix_zero(self.buf)
        if self.emulate is not None and self.device.type == "cuda":
            n, bw, lat = self.emulate
            self.emulate = (n, bw / 1.5, lat)
            efin = self._launch_reduce(lo, hi, packed)
            self.emulate = (n, bw, lat)
            return lambda: (efin(), (prefix0, operand))[1]
        return lambda: (prefix0, operand)

    def flush_correction(self) -> None:
        """Run the deferred record correction now (stream-ordered), if one is pending."""
        if self._pending is not None:
            rec, K, rows, delta = self._pending
            self._pending = None
            native().correct_records(rec, K, rows, delta)

    def pending_rows(self, out) -> bool:
        """Whether the deferred correction still has to write rows of RateResult ``out``."""
        if self._pending is None or out is None or getattr(out, "packed", None) is None:
            return False
        a, b = self._pending[2], out.packed
        a0, b0 = a.data_ptr(), b.data_ptr()
        return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()

    def merge(self, roster, overlap: Optional[Callable[[], None]] = None) -> None:
        """Combine every rank's window into the replicated roster (in place):
        messages -> all-reduce -> decode, pipelined over row buckets; the decode
        also writes the next window's common start.

        ``overlap``: independent main-stream work (the next window's schedule
        prepass, runtime/engine.py) enqueued once every bucket's all-reduce is in
        flight and before the first decode waits for one, so the collectives run
        under it instead of in front of it."""
        if self.world <= 1 and not self.force:
            self.windows += 1
            if overlap is not None:
                overlap()
            return
        packed = self._packed()
        msg = self.messages_packed if packed else self.messages
        dec = self.decode_packed if packed else self.decode
        if overlap is not None:
            self._ev("begin")
            launched = []
            for lo, hi in self.buckets():
                msg(roster, lo, hi)
                launched.append((lo, hi, self._launch_reduce(lo, hi, packed)))
            self._ev("messages")
            overlap()
            self._ev("overlap")
            for lo, hi, fin in launched:
                fin()
                self._ev("allreduce")
                dec(roster, lo, hi, into=self.start)
                self._ev("apply")
            self._synced = True
            self.windows += 1
            return
        pending = None  # (lo, hi, finisher) of the bucket whose reduce is in flight
        self._ev("begin")
        for lo, hi in self.buckets():
            msg(roster, lo, hi)
            self._ev("messages")
            fin = self._launch_reduce(lo, hi, packed)
            if pending is not None:
                plo, phi, pfin = pending
                pfin()
                self._ev("allreduce")
                dec(roster, plo, phi, into=self.start)
                self._ev("apply")
            pending = (lo, hi, fin)
        if pending is not None:
            plo, phi, pfin = pending
            pfin()
            self._ev("allreduce")
            dec(roster, plo, phi, into=self.start)
            self._ev("apply")
        self._synced = True
        self.windows += 1

    def clamp_hits(self) -> int:
        """Decoded tracks held at the precision floor since the last ``check`` (syncs)."""
        return int(self.clamps.item())

    def check(self) -> None:
        """Raise MergeClampError if any decode since the last check clamped (syncs);
        the counter restarts.  bench.py and runtime/rerate.py call it at the end of a
        run and before every checkpoint, as they check the executor's error flags."""
        n = self.clamp_hits()
        if n:
            self.clamps.zero_()
            raise MergeClampError("sweep merge: %d decoded track(s) had a merged precision at or below zero "
                                  "and were clamped (sigma x1000): the merged roster is not trustworthy"
                                  % n)

    def stage_ms(self) -> Dict[str, float]:
        """Per-stage main-stream time of the recorded merges (syncs; ``timing``):
        each event's time since the previous one, summed by stage name."""
        if not self._events:
            return {}
        torch.cuda.synchronize(self.device)
        out: Dict[str, float] = {}
        prev = None
        for name, e in self._events:
            if name != "begin" and prev is not None:
                out[name] = out.get(name, 0.0) + prev.elapsed_time(e)
            prev = e
        self._events.clear()
        return out


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def rate_window_dp(rater, merger: SweepMerger, roster, rec, K=None, out=None, check=True,
                   schedule=None):
    """One DP step: exact local rating of this rank's shard (``merger.sweeps``
    causal sweeps) + posterior merge."""
    merger.begin(roster)
    K = int(K or (rec.shape[1] - 2) // 2)
    if schedule is None and rec.is_cuda and merger.sweeps > 1:
        schedule = rater.schedule(rec, K, roster.num_players, tag="_dp")
    while True:
        res = rater.rate(roster, rec, K, out=out, check=check, schedule=schedule)
        merger.rated()
        if not merger.needs_resweep():
            break
        merger.resweep(roster)
        if schedule is not None:
            schedule.deps.zero_()  # the executor counted them up; links are reusable
        out = res
    merger.merge(roster)
    return res
