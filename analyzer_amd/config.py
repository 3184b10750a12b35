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
    # new: ENGINE=native keeps the player table resident on the device across batches
    resident: bool = True
    # new: the run is a benchmark -- synthetic telemetry may be persisted (worker.connect)
    synthetic_telemetry: bool = False
    # new: skip matches that already carry a rating (trueskill_quality set), so a
    # redelivery after commit-but-before-ack does not rate a match twice.  Off by
    # default: the reference re-rates redelivered matches (worker.py:122-129,194)
    skip_rated: bool = False

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
            resident=(env.get("RESIDENT") or "true") == "true",
            skip_rated=env.get("SKIP_RATED") == "true",
        )

    @property
    def failed_queue(self) -> str:
        return self.queue + "_failed"


@dataclass(frozen=True)
class EngineConfig:
    """Knobs of the MI355X rating engine (new; no reference counterpart)."""

    num_gpus: int = 1
    mode: str = "exact"           # exact | sweep
    window: int = 0               # matches per GPU per merge window (sweep mode); 0 = all
    comm_dtype: str = "fp32"      # fp32 | fp16 | bf16 compression of merge deltas
    checkpoint_every: int = 0     # windows between checkpoints (0 = off)
    checkpoint_dir: Optional[str] = None
    extra: Mapping[str, str] = field(default_factory=dict)

    @staticmethod
    def from_env(env: Mapping[str, str] = os.environ) -> "EngineConfig":
        return EngineConfig(
            num_gpus=int(_env(env, "NUM_GPUS") or 1),
            mode=_env(env, "MODE") or "exact",
            window=int(_env(env, "WINDOW") or 0),
            comm_dtype=_env(env, "COMM_DTYPE") or "fp32",
            checkpoint_every=int(_env(env, "CHECKPOINT_EVERY") or 0),
            checkpoint_dir=_env(env, "CHECKPOINT_DIR"),
        )
