"""Batched, exact TrueSkill rating of match streams (SURVEY K1-K6, A1 batched API).

``BatchRater.rate(roster, rec)`` is the tensor counterpart of calling
``rater.rate_match`` on every match of a stream in order
(/root/reference/worker.py:176-192 + rater.py:69-169):

* on a ROCm device it runs the schedule prepass (occurrence index per slot,
  csrc/kernels.hip ``launch_schedule``) and then the single-launch dataflow
  kernel that rates the whole stream in per-player chronological order;
* on the CPU it runs the C++ host mirror sequentially (fp64 by default), which
  is the semantic oracle for the device path.

The roster is updated in place.  Outputs are per match (quality, status) and
per slot ``[M, 2K]`` (shared mu/sigma and delta for ``participant``, mode
mu/sigma for ``participant_items``); NaN means "not written".
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, NamedTuple, Optional, Tuple

import torch

from ..config import MODES, N_TRACKS, EngineConfig, RaterConfig
from ..models.tiers import vst_table
from .native import native

# status codes (csrc/common.h)
RATED, AFK, INVALID_ROSTERS, UNSUPPORTED_MODE = 0, 1, 2, 3
ERR_SEED, ERR_SIGMA, ERR_EMPTY_ROSTER, ERR_NUMERIC, ERR_BAD_RECORD = 4, 5, 6, 7, 8
NOT_PROCESSED = 255
CTRL_WORDS = 52  # executor control words (csrc/dataflow.hip launch_rate)
STATUS_NAMES = {RATED: "rated", AFK: "afk", INVALID_ROSTERS: "invalid_rosters",
                UNSUPPORTED_MODE: "unsupported_mode", ERR_SEED: "error_seed",
                ERR_SIGMA: "error_sigma", ERR_EMPTY_ROSTER: "error_empty_roster",
                ERR_NUMERIC: "error_numeric", ERR_BAD_RECORD: "error_bad_record",
                NOT_PROCESSED: "not_processed"}
# the reference raises (and fails the whole batch) for these classes
ERROR_STATUSES = (ERR_SEED, ERR_SIGMA, ERR_EMPTY_ROSTER, ERR_NUMERIC, ERR_BAD_RECORD)


class NativeRateError(RuntimeError):
    pass


class Schedule(NamedTuple):
    # [M, 2K] int32 per slot: next match of the player (NO_MATCH: none) | HAS_PRED
    link: torch.Tensor
    # [M] int32.  Device: completion counters, zeroed by the prepass and counted up
    # by the executor as predecessors publish (a match is ready at the number of
    # its distinct players with HAS_PRED on their first slot).  Host mirror: that
    # number itself.
    deps: torch.Tensor

    NO_MATCH = 0x0FFFFFFF
    MATCH_MASK = 0x0FFFFFFF
    HAS_PRED = 1 << 30


@dataclass
class Roster:
    """Device-resident player table (structure of arrays, 128 B per player).

    ``state[p]`` = 8 granules of (mu, tag, sigma, tag): granule 0 the shared
    track, 1..6 the modes of ``config.MODES``, 7 spare; NaN mu = NULL.  Tags
    are owned by the dataflow kernel (csrc/kernels.hip); everything else writes
    0.  ``attrs[p]`` = (rank_points_ranked, rank_points_blitz, skill_tier, 0);
    NaN = NULL.  ``epoch`` numbers the device launches since the last tag reset
    (``None`` = tags of unknown origin, reset before the next device launch).
    """

    state: torch.Tensor
    attrs: torch.Tensor
    epoch: Optional[int] = None

    ROW = 32

    @property
    def num_players(self) -> int:
        return int(self.state.shape[0])

    @property
    def device(self) -> torch.device:
        return self.state.device

    @staticmethod
    def empty(num_players: int, device="cpu") -> "Roster":
        state = torch.zeros((num_players, 32), dtype=torch.float32, device=device)
        state[:, 0::2] = float("nan")
        attrs = torch.full((num_players, 4), float("nan"), dtype=torch.float32, device=device)
        attrs[:, 3] = 0.0
        return Roster(state, attrs, epoch=0)

    def tracks(self) -> torch.Tensor:
        """``[P, 8, 2]`` copy of (mu, sigma) per track."""
        return self.state.view(-1, 8, 4)[:, :, 0::2]

    def mu(self) -> torch.Tensor:
        return self.state[:, 0::4]

    def sigma(self) -> torch.Tensor:
        return self.state[:, 2::4]

    def track(self, name: str) -> torch.Tensor:
        """``[P, 2]`` (mu, sigma) of ``trueskill`` or ``trueskill_<mode>``."""
        idx = 0 if name in ("shared", "trueskill") else 1 + MODES.index(name.replace("trueskill_", ""))
        return self.state[:, 4 * idx:4 * idx + 3:2]

    def to(self, device) -> "Roster":
        return Roster(self.state.to(device), self.attrs.to(device), self.epoch)

    def clone(self) -> "Roster":
        return Roster(self.state.clone(), self.attrs.clone(), self.epoch)

    def next_epoch(self) -> int:
        """Epoch for the next device launch, resetting the tags when needed."""
        if self.epoch is None or self.epoch >= 255:
            native().reset_tags(self.state)
            self.epoch = 0
        self.epoch += 1
        return self.epoch


@dataclass
class RateResult:
    """Per-match outputs.  ``allocate`` packs every match into one 128-B aligned
    row of ``packed`` -- [s_mu | s_sig | delta | m_mu | m_sig][2K], quality, status
    byte -- so the executor writes each match with one full cache line; the fields
    below are strided views of it (csrc/common.h RateOut)."""

    quality: torch.Tensor   # [M]
    status: torch.Tensor    # [M] uint8
    s_mu: torch.Tensor      # [M, 2K]
    s_sig: torch.Tensor
    delta: torch.Tensor
    m_mu: torch.Tensor
    m_sig: torch.Tensor
    packed: Optional[torch.Tensor] = None  # [M, row] backing storage (None: separate arrays)

    FIELDS = ("quality", "status", "s_mu", "s_sig", "delta", "m_mu", "m_sig")

    @staticmethod
    def row_floats(K: int) -> int:
        return -(-(5 * 2 * K + 2) // 32) * 32

    @staticmethod
    def allocate(M: int, K: int, device, packed: bool = True) -> "RateResult":
        S = 2 * K
        if not packed:
            f = dict(dtype=torch.float32, device=device)
            return RateResult(torch.empty(M, **f), torch.empty(M, dtype=torch.uint8, device=device),
                              *(torch.empty((M, S), **f) for _ in range(5)))
        W = RateResult.row_floats(K)
        buf = torch.empty((M, W), dtype=torch.float32, device=device)
        slots = [buf[:, f * S:(f + 1) * S] for f in range(5)]
        status = buf.view(torch.uint8)[:, 4 * (5 * S + 1)]
        return RateResult(buf[:, 5 * S], status, *slots, packed=buf)

    @property
    def any_afk(self) -> torch.Tensor:
        """``participant_items.any_afk`` per match (True for AFK / invalid)."""
        return (self.status == AFK) | (self.status == INVALID_ROSTERS)

    def status_counts(self) -> Dict[str, int]:
        vals, counts = torch.unique(self.status.cpu(), return_counts=True)
        return {STATUS_NAMES.get(int(v), str(int(v))): int(c) for v, c in zip(vals, counts)}


class BatchRater:
    """Stateless-per-call batched rater with cached device workspaces."""

    def __init__(self, cfg: Optional[RaterConfig] = None, host_fp64: bool = True,
                 blocks: Optional[int] = None):
        self.cfg = cfg or RaterConfig.from_env()
        self.host_fp64 = host_fp64
        ecfg = EngineConfig.from_env()
        # persistent-grid size of the dataflow launch (4 waves per block): fixed by the
        # argument or ANA_RATE_BLOCKS, else chosen per launch (launch_blocks)
        self.fixed_blocks = int(blocks or ecfg.rate_blocks or 0)
        self.blocks = self.fixed_blocks or 512  # the full grid (aggregation tiles)
        self.knobs = ecfg.rate_knobs()  # executor / fused-telemetry tuning (csrc/bindings.cpp)
        # inline (fused) telemetry up to this many matches per launch, the MFMA kernel after
        # the rating above (scripts/tele_batch.py, profiles/r3/tele_fused_vs_separate_by_batch.log)
        self.tele_fuse_max = int(ecfg.tele_fuse_max)
        # ANA_RATE_CHUNK (tuning): cap on the matches per ticket of a window launch (8-64;
        # default per team size, chunk_len)
        self.chunk_cap = int(os.environ.get("ANA_RATE_CHUNK") or 0)
        self._vst: Dict[str, torch.Tensor] = {}
        self._ws: Dict[Tuple[str, str], torch.Tensor] = {}

    @staticmethod
    def has_telemetry(telemetry) -> bool:
        """One definition of "this launch aggregates telemetry" for every caller
        that sizes chunks (rate(), runtime/engine.py's tail signal)."""
        return telemetry is not None and telemetry[0].numel() > 0

    def tiles(self, telemetry, M: int) -> bool:
        """Does a launch of M matches with ``telemetry`` aggregate in MFMA tiles of
        its own waves (ANA_TELE_ROLE >= 0), which need the full grid and 64-match
        chunks?  Inline aggregation (the default) and launches past
        ``tele_fuse_max`` (aggregated by the kernel after the rating) do not."""
        return self.has_telemetry(telemetry) and self.knobs[5] >= 0

    def fuses(self, telemetry, M: int) -> bool:
        """Is ``telemetry`` aggregated inside the rating launch of M matches?  Tiles
        always are; inline aggregation up to ``tele_fuse_max`` matches.  Above it the
        standalone MFMA kernel runs after the rating on the same stream: inline costs
        each rating iteration its event loads and LDS adds, which a latency-bound
        window pays on every dependency level (10M 3v3: 11.1 ms fused vs 9.9 ms
        separate), while a worker batch is launch-bound (500 matches: 44 vs 80 us)."""
        return self.has_telemetry(telemetry) and (self.knobs[5] >= 0 or M <= self.tele_fuse_max)

    def launch_blocks(self, K: int = 3, roster_bytes: int = 0) -> int:
        """Workgroups of a window launch: 256 (one wave per SIMD) over a roster that fits
        the 256-MB Infinity Cache, else 512.  Measured per workload on MI355X
        (profiles/r5/executor_grid.log, 256 vs 512): 3v3 over 1M players 6.56 vs 6.65 ms
        per 10M window, config 2 step 7.95 vs 8.01, config 4 8.85 vs 9.35, skewed windows
        -4.5 / -6 %; 10M players (config 5, 1.28-GB roster: the gathers miss to HBM and
        need the waves) 13.05 vs 11.73.  4v4 and 5v5 took 512 until the one-held-chunk
        executor: since then 256 wins for them too -- 4v4 (10M window) 9.29-9.56 vs
        10.77-10.80 ms per step, config 3 with 32-match chunks 14.36-14.48 vs 15.43-15.51
        (profiles/r6/wide_teams_grid_chunk.log)."""
        if self.fixed_blocks:
            return self.fixed_blocks
        return 256 if roster_bytes <= (256 << 20) else 512

    def chunk_len(self, M: int, telemetry: bool = False, blocks: Optional[int] = None, K: int = 3) -> int:
        """Matches per executor ticket: 64 (one per lane) for windows -- 32 for 5v5 --,
        shorter (8-32, a power of two) when such chunks would leave the full grid
        (``4 * self.blocks`` waves) short of work.  A wave rates 64/G matches per
        iteration, so a 500-match micro-batch in 64-match chunks runs 8 waves x 8
        dependent iterations; in 8-match chunks it runs 63 waves x 1.  5v5 windows are
        ~3,000 dependency levels of ~4k matches: a wave holding 32 claims closer to the
        frontier (config 3 18.5-18.9 -> 15.4-15.5 ms per step at 512 workgroups; 16:
        22.8; 3v3 and 4v4 lose with 32: config 2 8.45, config 5 13.96, 4v4 9.74-9.93 vs
        9.29-9.56 ms, profiles/r6/wide_teams_grid_chunk.log).  ``ANA_RATE_CHUNK`` caps it."""
        if telemetry:
            return 64
        cap = self.chunk_cap if self.chunk_cap > 0 else (32 if K >= 5 else 64)
        need = -(-M // (4 * (blocks or self.blocks)))  # matches per wave at the full grid
        cl = 8
        while cl < need and cl < 64:
            cl *= 2
        return max(8, min(cl, cap))

    def grid_blocks(self, M: int, telemetry: bool = False, blocks: Optional[int] = None, K: int = 3) -> int:
        """Persistent-grid size for a window of M matches: ``blocks`` (launch_blocks),
        but no more than one wave per chunk (``chunk_len``) -- a micro-batch of 500
        matches needs 63 waves, not 2048 (the extra workgroups only cost launch and exit
        time).  Fused telemetry tiles keep the full grid (they need the waves)."""
        if telemetry:
            return self.blocks
        b = blocks or self.blocks
        chunks = -(-M // self.chunk_len(M, blocks=b, K=K))
        return max(1, min(b, -(-chunks // 4)))

    # ------------------------------------------------------------- buffers
    def vst(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._vst:
            self._vst[key] = torch.tensor(vst_table(), dtype=torch.float32, device=device)
        return self._vst[key]

    def _buffer(self, device, name: str, numel: int, dtype) -> torch.Tensor:
        key = (str(device), name)
        buf = self._ws.get(key)
        if buf is None or buf.numel() < numel or buf.dtype != dtype:
            buf = torch.empty(int(numel), dtype=dtype, device=device)
            self._ws[key] = buf
        return buf[:numel]

    def _ctrl(self, device) -> torch.Tensor:
        """The executor's control words (csrc/dataflow.hip launch_rate): [0..15]
        per launch (zeroed before each), [16..18] sticky OR of the error flags
        over every launch since ``clear_sticky``."""
        key = (str(device), "ctrl")
        buf = self._ws.get(key)
        if buf is None:
            buf = torch.zeros(CTRL_WORDS, dtype=torch.int32, device=device)
            self._ws[key] = buf
        return buf

    # ------------------------------------------------------------- schedule
    def schedule(self, rec: torch.Tensor, K: int, num_players: int,
                 tag: str = "", zero_ctrl: bool = False,
                 epoch_bump: Optional[torch.Tensor] = None, sort_nt: int = -1) -> Schedule:
        """Dependency structure of a window (K5): per slot the match of its
        player's next occurrence and whether it occurred earlier (``link``), and
        per match the completion counter ``deps`` (see ``Schedule``).  The device
        rate launch counts ``deps`` up, so a schedule is single-use there.
        ``tag`` selects a separate buffer set (to prepare the next window while the
        current one is being rated).  ``zero_ctrl`` (used by ``rate`` only): the
        schedule also zeroes the executor's control words for the launch that
        follows it on the same stream -- never from a side stream, where a rate
        launch may be using them.  ``epoch_bump``: a device int32 launch epoch
        (graph replays) the schedule increments, saving the bump its own dispatch.
        ``sort_nt``: non-temporal accesses of the radix sort (0 none, 1 all, 2 loads
        only; -1: ANA_SORT_NT or none) -- ANA_SORT_NT, when set, wins."""
        M = rec.shape[0]
        dev = rec.device
        link = self._buffer(dev, "link" + tag, M * 2 * K, torch.int32).view(M, 2 * K)
        deps = self._buffer(dev, "deps" + tag, M, torch.int32)
        if rec.is_cuda:
            nbytes = native().schedule_workspace_bytes(M * 2 * K, num_players)
            ws = self._buffer(dev, "sched_ws", nbytes, torch.uint8)
            ctrl = self._ctrl(dev)
        else:
            ws = torch.empty(0, dtype=torch.uint8)
            ctrl = torch.empty(0, dtype=torch.int32)
        bump = epoch_bump.data_ptr() if epoch_bump is not None and rec.is_cuda else 0
        native().schedule(rec, K, num_players, link, deps, ws, ctrl, bool(zero_ctrl and rec.is_cuda),
                          bump, int(sort_nt))
        return Schedule(link, deps)

    # ----------------------------------------------------------------- rate
    def rate(self, roster: Roster, rec: torch.Tensor, K: Optional[int] = None,
             out: Optional[RateResult] = None, first_prior: Optional[torch.Tensor] = None,
             check: bool = True, schedule: Optional[Schedule] = None,
             telemetry=None, progress=None, epoch_dev: Optional[torch.Tensor] = None) -> RateResult:
        """Rate every match of ``rec`` in order, updating ``roster`` in place.

        ``telemetry`` = (evoff [M+1] int64, events [E,2] int32, stats [M,2K,8] f32):
        per-participant telemetry is aggregated into ``stats`` -- in the same launch
        up to ``tele_fuse_max`` matches (K8 fused streaming mode: each lane group folds
        the events of the match it rates), by the MFMA kernel right after it above
        (``fuses``).
        ``progress`` = (signal address, launch number, chunk index): the tail
        signal of runtime/engine.py (device only).  ``epoch_dev``: a device int32
        tensor holding the launch epoch (graph replays, ops/graph.py), bumped by
        one on the device before the launch reads it; the roster's host-side
        epoch is then left alone."""
        K = int(K or (rec.shape[1] - 2) // 2)
        M = int(rec.shape[0])
        dev = rec.device
        if roster.device != dev:
            raise ValueError("roster is on %s but the stream is on %s" % (roster.device, dev))
        if out is None:
            out = RateResult.allocate(M, K, dev)
        P = roster.num_players
        cfg = self.cfg
        record = first_prior is not None
        fp = first_prior if record else torch.empty(0, dtype=torch.float32, device=dev)
        if dev.type == "cuda":
            ctrl_ready = schedule is None  # the schedule below zeroes ctrl on this stream
            if schedule is None:  # ... and bumps a device epoch
                schedule = self.schedule(rec, K, P, zero_ctrl=True, epoch_bump=epoch_dev)
            elif epoch_dev is not None:
                native().epoch_bump(epoch_dev)
            link, deps = schedule
            ctrl = self._ctrl(dev)
            epoch = roster.next_epoch() if epoch_dev is None else 1
        else:
            link = deps = ctrl = torch.empty(0, dtype=torch.int32)
            epoch = 1
            ctrl_ready = False
        blocks = self.launch_blocks(K, roster.state.numel() * roster.state.element_size())
        # aggregation tiles need the full grid and whole chunks; inline aggregation
        # (ANA_TELE_ROLE < 0: each lane group folds its own match's events) does not
        tiles = self.tiles(telemetry, M)
        after = None
        if self.has_telemetry(telemetry) and not self.fuses(telemetry, M) and dev.type == "cuda":
            after, telemetry = telemetry, None  # the MFMA kernel after the rating (fuses())
        tele = self.has_telemetry(telemetry)
        if not tele:
            none = torch.empty(0, dtype=torch.int64, device=dev)
            telemetry = (none, none.to(torch.int32), none.to(torch.float32))
        native().rate(rec, K, link, deps, roster.state, roster.attrs, fp, out.quality, out.status,
                      out.s_mu, out.s_sig, out.delta, out.m_mu, out.m_sig, ctrl, self.vst(dev),
                      float(cfg.beta) ** 2, float(cfg.tau) ** 2, float(cfg.unknown_player_sigma),
                      record, self.grid_blocks(M, tiles, blocks, K), epoch,
                      self.host_fp64, *telemetry,
                      *(progress if progress is not None and dev.type == "cuda" else (0, 0, 0)),
                      epoch_dev.data_ptr() if epoch_dev is not None and dev.type == "cuda" else 0,
                      self.chunk_len(M, tiles, blocks, K), ctrl_ready, self.knobs)
        if after is not None:
            # same stream, after the rating; malformed events count into ctrl[13] as in
            # the fused launch (zeroed by this launch, read by telemetry_errors)
            evoff, events, stats = after
            native().telemetry(evoff, events, K, stats, ctrl[13:14])
        if check and dev.type == "cuda":
            self.check_errors(dev)
        return out

    def stale_retries(self, device) -> int:
        """Granule reads of the last launch that found their predecessor's write not
        yet landed and were retried (diagnostics; syncs)."""
        return int(self._ctrl(device)[14].item())

    def iterations(self, device) -> int:
        """Wave iterations of the last executor launch (diagnostics; syncs)."""
        return int(self._ctrl(device)[15].item())

    def handoffs(self, device) -> Tuple[int, int]:
        """(local, global) dependency hand-offs of the last launch: successors
        released through the producing wave's LDS counters vs the global ones."""
        c = self._ctrl(device)[26:28].cpu()
        return int(c[0]), int(c[1])

    def diag(self, device) -> Dict[str, float]:
        """Timing-build statistics of the last launch (ANA_RATE_DIAG=1; syncs).
        Over the wave iterations that rated something: the mean time from the
        top of the loop to the iteration's one wait (issue), in the wait, and
        after it (rating, publish, bookkeeping), in microseconds."""
        c = [int(x) & 0xffffffff for x in self._ctrl(device).cpu().tolist()]
        u64 = lambda i: c[i] | (c[i + 1] << 32)
        worked = c[20]
        per = (lambda t: t * 0.01 / worked) if worked else (lambda t: 0.0)  # 100 MHz ticks -> us
        return {"wave_iterations": c[15], "worked_iterations": worked, "groups_assigned": c[21],
                "matches_per_worked_iteration": c[21] / worked if worked else 0.0,
                "issue_us": per(u64(22)), "wait_us": per(u64(24)), "after_us": per(u64(28)),
                # the after phase split: priors + team sums, coefficients + update,
                # publish (granules + hand-off), output records + bookkeeping
                "after_prior_us": per(u64(32)), "after_update_us": per(u64(34)),
                "after_publish_us": per(u64(36)), "after_rest_us": per(u64(38)),
                # the issue phase split: chunk staging + readiness, assignment (pick
                # list), this batch's loads, next polls + ticket
                "issue_ready_us": per(u64(40)), "issue_assign_us": per(u64(42)),
                "issue_loads_us": per(u64(44)), "issue_polls_us": per(u64(46)),
                "local_handoffs": c[26], "global_handoffs": c[27],
                # held matches one dependency short of ready / pending, per worked iteration
                "near_ready_per_worked_iteration": c[30] / worked if worked else 0.0,
                "pending_per_worked_iteration": c[31] / worked if worked else 0.0,
                "stale_retries": c[14]}

    def telemetry_errors(self, device) -> int:
        """Malformed telemetry events seen by the last fused launch (syncs)."""
        return int(self._ctrl(device)[13].item())

    def error_flags(self, device) -> torch.Tensor:
        """Device tensor [schedule overflow, timeout, protocol] of the last launch (no sync)."""
        return self._ctrl(device)[0:3]

    def sticky_flags(self, device) -> torch.Tensor:
        """Device tensor [schedule, timeout, protocol]: OR over every launch since
        the last ``clear_sticky`` (no sync) -- a window pipeline checks this once
        instead of after each launch, without losing a middle window's failure."""
        return self._ctrl(device)[16:19]

    def clear_sticky(self, device) -> None:
        self._ctrl(device)[16:19].zero_()

    def check_errors(self, device, sticky: bool = False) -> None:
        self.raise_flags((self.sticky_flags(device) if sticky else self.error_flags(device)).cpu())

    @staticmethod
    def raise_flags(flags: torch.Tensor) -> None:
        """Raise on host copies of ``error_flags`` / ``sticky_flags``."""
        if int(flags[0]):
            raise NativeRateError("schedule prepass failed (flag %d)" % int(flags[0]))
        if int(flags[1]):
            raise NativeRateError("dataflow rating timed out (a dependency never resolved)")
        if int(flags[2]):
            raise NativeRateError("dataflow race detected: a player's granule was written by a "
                                  "later match before an earlier one read it")


def rate_stream(roster: Roster, rec: torch.Tensor, K: Optional[int] = None,
                cfg: Optional[RaterConfig] = None) -> RateResult:
    """Convenience wrapper: ``BatchRater(cfg).rate(roster, rec, K)``."""
    return BatchRater(cfg).rate(roster, rec, K)


__all__ = ["Roster", "RateResult", "BatchRater", "rate_stream", "STATUS_NAMES", "N_TRACKS"]
