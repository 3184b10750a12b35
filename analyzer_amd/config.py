"""Environment-variable configuration (SURVEY W1, R1 and §5 "Config / flags").

Names and defaults match the reference exactly:

* worker: /root/reference/worker.py:16-27 (``RABBITMQ_URI``, ``DATABASE_URI``,
  ``BATCHSIZE``, ``CHUNKSIZE``, ``IDLE_TIMEOUT``, ``QUEUE``, ``DOCRUNCHMATCH``,
  ``CRUNCH_QUEUE``, ``DOTELESUCKMATCH``, ``TELESUCK_QUEUE``, ``DOSEWMATCH``,
  ``SEW_QUEUE``); boolean flags are on only for the literal string ``"true"``.
* rater: /root/reference/rater.py:10-11 (``UNKNOWN_PLAYER_SIGMA``, ``TAU``).

Differences (documented, deliberate): ``DATABASE_URI`` is not required at import
time -- without it the worker uses the in-process store (the reference raises
``KeyError`` on import, which makes ``import worker`` impossible in tests).
New knobs for the MI355X engine are read here too, once, into frozen dataclasses.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Mapping, Optional

# model constants fixed by the reference (rater.py:30-37)
BETA = 10.0 / 30 * 3000          # = 1000.0
ENV_MU = 1500.0
ENV_SIGMA = 1000.0
DRAW_PROBABILITY = 0.0

# game modes the rater understands, in device track order (track 0 = shared)
MODES = ("casual", "ranked", "blitz", "br", "5v5_casual", "5v5_ranked")
TRACK_COLUMNS = ("trueskill",) + tuple("trueskill_" + m for m in MODES)
N_TRACKS = len(TRACK_COLUMNS)    # 7
MODE_UNSUPPORTED = 255


def _env(env: Mapping[str, str], key: str) -> Optional[str]:
    v = env.get(key)
    return v if v else None


def _tristate(v: Optional[str]) -> Optional[bool]:
    """'1'/'0' -> True/False; unset, empty or 'auto' -> None."""
    if v is None or v == "" or v.lower() == "auto":
        return None
    return v != "0"


def _resident_default(env: Mapping[str, str]) -> bool:
    v = env.get("RESIDENT")
    if v:
        # several replicas on one store (runtime/replicas.py sets REPLICA, a tcp:// broker):
        # a resident roster would keep rating from its own cached rows and overwrite the
        # other replicas' commits -- the device rows are re-read from the store per batch
        if v == "true" and (env.get("REPLICA") or (env.get("RABBITMQ_URI") or "").startswith("tcp://")):
            return False
        return v == "true"
    uri = env.get("DATABASE_URI") or ""
    return uri == "" or uri.startswith(("memory:", "columnar:"))


@dataclass(frozen=True)
class RaterConfig:
    unknown_player_sigma: int = 500
    tau: float = 1000 / 100.0
    beta: float = BETA
    backend: str = "closed"      # closed (fp64 closed form) | ep | mpmath

    @staticmethod
    def from_env(env: Mapping[str, str] = os.environ) -> "RaterConfig":
        return RaterConfig(
            unknown_player_sigma=int(_env(env, "UNKNOWN_PLAYER_SIGMA") or 500),
            tau=float(_env(env, "TAU") or 1000 / 100.0),
            backend=_env(env, "RATER_BACKEND") or "closed",
        )


@dataclass(frozen=True)
class WorkerConfig:
    rabbitmq_uri: str = "amqp://localhost"
    database_uri: Optional[str] = None
    batchsize: int = 500
    chunksize: int = 100
    idle_timeout: float = 1.0
    queue: str = "analyze"
    docrunchmatch: bool = False
    crunch_queue: str = "crunch_global"
    dotelesuckmatch: bool = False
    telesuck_queue: str = "telesuck"
    dosewmatch: bool = False
    sew_queue: str = "sew"
    # new: which rating path processes a batch (python | native)
    engine: str = "python"
    # new: quarantine only the failing matches of a batch (false: fail the whole batch)
    quarantine: bool = True
    # new: aggregate per-participant telemetry (participant_stats) in the rating launch
    dotelemetry: bool = False
    telemetry_events: str = "100,300"
    # new: ENGINE=native keeps the player table resident on the device across batches.
    # Default (RESIDENT unset): on for the in-process stores only -- a resident roster
    # never re-reads the store, so with a shared SQL database another worker replica's
    # writes would be overwritten with stale ratings.  RESIDENT=true opts in anyway.
    resident: bool = True
    # new: the run is a benchmark -- synthetic telemetry may be persisted (worker.connect)
    synthetic_telemetry: bool = False
    # new: DOTELEMETRY event source -- an ANATEL01 file of downloaded events keyed by
    # match api id (ops/telemetry.TelemetrySource); unset = synthetic events
    telemetry_source: Optional[str] = None
    # new: skip matches that already carry a rating (trueskill_quality set), so a
    # redelivery after commit-but-before-ack does not rate a match twice.  Off by
    # default: the reference re-rates redelivered matches (worker.py:122-129,194)
    skip_rated: bool = False
    # new: keep two batches in flight on the columnar native path (runtime/worker.py
    # "pipelined batches"); prefetch becomes 2 x BATCHSIZE.  Off by default: at
    # BATCHSIZE=500 the device part of a batch is ~10 us of a ~1 ms host-bound batch,
    # and the second batch's bookkeeping measured 3-6 % slower (profiles/r3/worker_*)
    pipeline: bool = False
    # new: fault injection -- these match api ids fail to rate as if their
    # numerics broke: quarantined (QUARANTINE=true) or failing their batch (false)
    fault_poison: frozenset = frozenset()
    # new: fault injection -- the process dies (exit 17) when a batch arrives after this
    # many processed batches, holding its unacknowledged deliveries (replica death:
    # the broker redelivers them to the other replicas, runtime/replicas.py)
    fault_exit_after: int = 0
    # new: replicas on one SQL store (runtime/store.py versioned player rows): a batch whose
    # compare-and-set player writes find a row another replica changed since it was read is
    # rolled back and rated again from fresh rows, up to this many times (then it fails)
    cas_retries: int = 50

    @staticmethod
    def from_env(env: Mapping[str, str] = os.environ) -> "WorkerConfig":
        return WorkerConfig(
            rabbitmq_uri=_env(env, "RABBITMQ_URI") or "amqp://localhost",
            database_uri=_env(env, "DATABASE_URI"),
            batchsize=int(_env(env, "BATCHSIZE") or 500),
            chunksize=int(_env(env, "CHUNKSIZE") or 100),
            idle_timeout=float(_env(env, "IDLE_TIMEOUT") or 1),
            queue=_env(env, "QUEUE") or "analyze",
            docrunchmatch=env.get("DOCRUNCHMATCH") == "true",
            crunch_queue=_env(env, "CRUNCH_QUEUE") or "crunch_global",
            dotelesuckmatch=env.get("DOTELESUCKMATCH") == "true",
            telesuck_queue=_env(env, "TELESUCK_QUEUE") or "telesuck",
            dosewmatch=env.get("DOSEWMATCH") == "true",
            sew_queue=_env(env, "SEW_QUEUE") or "sew",
            engine=_env(env, "ENGINE") or "python",
            quarantine=(env.get("QUARANTINE") or "true") == "true",
            dotelemetry=env.get("DOTELEMETRY") == "true",
            telemetry_events=_env(env, "TELEMETRY_EVENTS") or "100,300",
            synthetic_telemetry=env.get("SYNTHETIC_TELEMETRY") == "true",
            telemetry_source=_env(env, "TELEMETRY_SOURCE"),
            resident=_resident_default(env),
            skip_rated=env.get("SKIP_RATED") == "true",
            pipeline=env.get("PIPELINE") == "true",
            fault_poison=frozenset(x for x in (env.get("FAULT_POISON") or "").split(",") if x),
            fault_exit_after=int(env.get("FAULT_EXIT_AFTER") or 0),
            cas_retries=int(env.get("CAS_RETRIES") or 50),
        )

    @property
    def failed_queue(self) -> str:
        return self.queue + "_failed"


@dataclass(frozen=True)
class EngineConfig:
    """Knobs of the MI355X rating engine (new; no reference counterpart), read
    once from the environment.  The Python-side consumers take their defaults
    from here (``EngineConfig.from_env()``); the knobs the native extension reads
    at launch time are listed in ``NATIVE_KNOBS`` with what they do.

    ======================  ========  =============================================
    variable                default   consumer
    ======================  ========  =============================================
    ANA_RATE_BLOCKS         0         persistent grid of a window launch (0: 256 or 512 by workload, ops/rate.py)
    ANA_PREPASS_AT          0.7       tail overlap point of the next prepass (runtime/engine.py; 0.9 for
                                      1v1-4v4 windows between DP merges)
    ANA_PREPASS_CUS         0         CU-masked prepass stream, 0 = off (runtime/engine.py)
    ANA_PREPASS_SERIAL      auto      1 prepass on the main stream, 0 tail overlap; auto: serial
                                      for K <= 4 without DP merges, overlap otherwise (runtime/engine.py)
    ANA_ROSTER_WARM         auto      read the roster once in front of each window's rating launch, so
                                      its rows come from the Infinity Cache (runtime/engine.py); auto =
                                      on between DP merges (short windows: k = 8 forced merges 9.30 vs
                                      9.53 ms), off for whole windows (8.02 either way)
    ANA_MERGE_BUCKET_MB     64        sweep-merge bucket size (parallel/sweep.py)
    ANA_DP_SERIAL_AR_US     40        DP with N > 1 ranks: the next prepass runs beside the merge when one
                                      merge-sized all-reduce (timed when the pipeline is built, max over
                                      ranks) takes longer than this, else in the rating's tail
                                      (runtime/engine.py probe_placement)
    COMM_DTYPE              (unset)   sweep-merge message precision (bench.py, rerate): unset = fp16 for one
                                      sweep (BASELINE config 5: fp16 moments), fp32 for causal re-sweeps
    SWEEPS                  1         causal sweeps per window (bench.py, rerate)
    ANA_DIST_BACKEND        nccl      process group backend (gloo: N ranks on one GPU)
    CHECKPOINT_DIR / _EVERY -- / 1    re-rate checkpoints (runtime/rerate.py)
    ANA_TRACE               0         roctx ranges + Chrome trace (utils/trace.py)
    ANA_CHECK_ROUNDS        0         exact DP race detector: rounds share no player (parallel/exact_dp.py)
    ANA_RATE_IDLE           0         executor: max s_sleep rounds of an idle wave (<= 0: none)
    ANA_RATE_LOCAL          1         executor: LDS hand-off of successors the producing wave holds (0 = off; 1v1-3v3)
    ANA_RATE_DIAG           0         executor timing build: per-phase clocks in ctrl[20..47] (ops/rate.diag)
    ANA_RATE_TIGHT          -1        executor: 2K lanes per match instead of the next power of two (-1 auto)
    ANA_TELE_FUSED_TAIL     0         fused telemetry only after the executor's chunks are drained
    ANA_TELE_ROLE           -1        fused telemetry: -1 = inline, each lane group folds the events of
                                      the match it rates (11.4 ms per config 4 step); N > 0 = one wave in
                                      N aggregates MFMA tiles from the start (N = 2: 11.7); 0 = idle waves.
                                      All slower than the separate kernel on 10M windows (10.1)
    ANA_TELE_FUSE_MAX       262144    inline (fused) telemetry up to this many matches per launch; larger
                                      launches rate, then run the MFMA kernel (ops/rate.py; crossover
                                      measured by scripts/tele_batch.py: fused 0.55x separate at 500
                                      matches, 0.96x at 100k, 1.05x at 1M)
    ======================  ========  =============================================

    The executor / fused-telemetry knobs reach the launch as ``BatchRater.knobs``
    (read once per BatchRater, passed to csrc/bindings.cpp ``rate``).
    """

    rate_blocks: int = 0  # 0: per launch (ops/rate.py launch_blocks)
    prepass_at: float = 0.7
    prepass_at_set: bool = False  # ANA_PREPASS_AT given explicitly (else the engine picks per mode)
    prepass_cus: int = 0
    prepass_exclusive: bool = False  # with prepass_cus: the executor gets the other CUs
    prepass_serial: Optional[bool] = None  # None = auto (WindowPipeline.serial_prepass)
    roster_warm: Optional[bool] = None  # None = auto (WindowPipeline)
    merge_bucket_mb: float = 64.0
    comm_dtype: str = ""  # "" = by sweeps (runtime/rerate.py default_comm_dtype)
    sweeps: int = 1
    dist_backend: str = "nccl"
    checkpoint_every: int = 1
    checkpoint_dir: Optional[str] = None
    trace: bool = False
    check_rounds: bool = False
    rate_idle: int = 0
    # LDS hand-off of successors the producing wave holds: off since round 5 -- at one wave
    # per SIMD with idle waves re-polling at once, the global counter path is as fast on a
    # serial chain and faster everywhere else (config 2 -0.03 ms, config 3 -0.13, quadratic /
    # cubic skew -3.8 / -3.3 %; config 5 +0.04, noise; profiles/r5/local_handoff_off.log)
    rate_local: int = 1
    rate_diag: int = 0
    rate_tight: int = -1
    tele_fused_tail: int = 0
    tele_role: int = -1
    tele_fuse_max: int = 262_144

    # kernel-implementation A/B switches read by the native extension itself
    # (csrc/telemetry.hip, kernels.hip, radix_sort.hip) -- experiments, not tuning
    NATIVE_KNOBS = {
        "ANA_TELE_IMPL": "telemetry aggregation: 1 one-hot MFMA GEMM (default), 0 LDS atomics",
        "ANA_SCHED_SMALL": "micro-batch schedule: hash lists (default) or bitonic sort",
        "ANA_SORT_RB / ANA_SORT_NT": "radix-sort tile rows / non-temporal loads (tuning)",
        "ANA_SCHED_RUNS": "last schedule pass: run-end table (1, default) or digit offsets + fix-up (0)",
    }

    def rate_knobs(self) -> list:
        """[idle, local, diag, tight, tele_fused_tail, tele_role] for the native launch."""
        return [self.rate_idle, self.rate_local, self.rate_diag, self.rate_tight, self.tele_fused_tail,
                self.tele_role]

    @staticmethod
    def from_env(env: Mapping[str, str] = os.environ) -> "EngineConfig":
        return EngineConfig(
            rate_blocks=int(_env(env, "ANA_RATE_BLOCKS") or 0),
            prepass_at=float(_env(env, "ANA_PREPASS_AT") or 0.7) if env.get("ANA_PREPASS_AT") != "0" else 0.0,
            prepass_at_set=bool(env.get("ANA_PREPASS_AT")),
            prepass_cus=int(_env(env, "ANA_PREPASS_CUS") or 0),
            prepass_exclusive=env.get("ANA_PREPASS_EXCLUSIVE", "0") not in ("", "0", "false"),
            prepass_serial=_tristate(env.get("ANA_PREPASS_SERIAL")),
            roster_warm=_tristate(env.get("ANA_ROSTER_WARM")),
            merge_bucket_mb=float(_env(env, "ANA_MERGE_BUCKET_MB") or 64),
            comm_dtype=_env(env, "COMM_DTYPE") or "",
            sweeps=int(_env(env, "SWEEPS") or 1),
            dist_backend=_env(env, "ANA_DIST_BACKEND") or "nccl",
            checkpoint_every=int(_env(env, "CHECKPOINT_EVERY") or 1),
            checkpoint_dir=_env(env, "CHECKPOINT_DIR"),
            trace=(env.get("ANA_TRACE") or "0") not in ("", "0"),
            check_rounds=(env.get("ANA_CHECK_ROUNDS") or "0") not in ("", "0"),
            rate_idle=int(_env(env, "ANA_RATE_IDLE") or 0),
            rate_local=int(_env(env, "ANA_RATE_LOCAL") or 1),
            rate_diag=int(_env(env, "ANA_RATE_DIAG") or 0),
            rate_tight=int(_env(env, "ANA_RATE_TIGHT") or -1),
            tele_fused_tail=int(_env(env, "ANA_TELE_FUSED_TAIL") or 0),
            tele_role=int(_env(env, "ANA_TELE_ROLE") or -1),
            tele_fuse_max=int(_env(env, "ANA_TELE_FUSE_MAX") or 262_144),
        )
