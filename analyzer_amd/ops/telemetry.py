"""Per-event telemetry aggregation (BASELINE config 4).

The reference forwards each match's telemetry asset URL to a downstream
"telesuck" queue (/root/reference/worker.py:148-161) and maps, but never fills,
``participant_stats`` (worker.py:75-78).  Here the telemetry itself is
aggregated on the device into one stat vector per participant slot,
``stats[M, 2K, 8]`` = (kills, deaths, assists, damage, gold, farm, healing,
events) -- aligned with the rating outputs ``[M, 2K]``:

* ``aggregate`` runs the standalone kernel (one wave per span of matches, a
  one-hot GEMM on the matrix cores -- or LDS float atomics, ANA_TELE_IMPL=0 --
  and coalesced stat stores; csrc/telemetry.hip, telemetry_dev.h);
* ``BatchRater.rate(..., telemetry=(evoff, events, stats))`` runs it INSIDE the
  dataflow launch: waves with no ready match aggregate telemetry tiles instead
  of sleeping, so a latency-bound rating absorbs the bandwidth-bound
  aggregation (the fused streaming mode).

Events are 8-B records (slot | type << 8 | 16-bit match tag << 16, value bits)
grouped by match with CSR offsets ``evoff[M+1]`` (layout: csrc/telemetry_core.h).  ``make_telemetry`` generates them with the
counter RNG (deterministic per global match index, device or host).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import NamedTuple, Optional

import numpy as np
import torch

from .native import native

STAT_NAMES = ("kills", "deaths", "assists", "damage", "gold", "farm", "healing", "events")
EVENT_TYPES = ("kill", "death", "assist", "damage", "gold", "farm", "heal", "other")


@dataclass(frozen=True)
class TelemetrySpec:
    seed: int = 77
    min_events: int = 100
    max_events: int = 300


class Telemetry(NamedTuple):
    evoff: torch.Tensor   # [M + 1] int64
    events: torch.Tensor  # [E, 2] int32: slot | type << 8 | match tag << 16, value bits

    @property
    def num_events(self) -> int:
        return int(self.events.shape[0])


def make_telemetry(spec: TelemetrySpec, rec: torch.Tensor, K: int, base: int = 0) -> Telemetry:
    """Synthetic telemetry for the matches of ``rec`` (global indices base..)."""
    M = int(rec.shape[0])
    counts = native().gen_event_counts(M, spec.seed, spec.min_events, spec.max_events, base, rec.device)
    evoff = torch.zeros(M + 1, dtype=torch.int64, device=rec.device)
    torch.cumsum(counts, 0, out=evoff[1:])
    E = int(evoff[-1].item())
    events = torch.empty((E, 2), dtype=torch.int32, device=rec.device)
    native().gen_events(rec, K, evoff, spec.seed, spec.min_events, spec.max_events, base, events)
    return Telemetry(evoff, events)


def allocate_stats(M: int, K: int, device) -> torch.Tensor:
    return torch.zeros((M, 2 * K, len(STAT_NAMES)), dtype=torch.float32, device=device)


def aggregate(tel: Telemetry, K: int, stats: Optional[torch.Tensor] = None,
              bad: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Standalone aggregation into ``stats [M, 2K, 8]``."""
    M = tel.evoff.numel() - 1
    dev = tel.events.device
    if stats is None:
        stats = allocate_stats(M, K, dev)
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
    native().telemetry(tel.evoff, tel.events, K, stats, bad)
    return stats


def aggregate_reference(tel: Telemetry, K: int) -> np.ndarray:
    """fp64 numpy oracle of the aggregation (well-formed events only)."""
    ev = tel.events.cpu().numpy()
    M = tel.evoff.numel() - 1
    out = np.zeros((M, 2 * K, len(STAT_NAMES)), dtype=np.float64)
    if ev.shape[0] == 0:
        return out
    m = np.repeat(np.arange(M, dtype=np.int64), np.diff(tel.evoff.cpu().numpy()))  # CSR position
    slot = ev[:, 0] & 0xFF
    typ = (ev[:, 0] >> 8) & 0xFF
    val = ev[:, 1].view(np.float32).astype(np.float64)
    add = np.where(typ <= 2, 1.0, val)
    feat = np.where(typ <= 6, typ, -1)
    ok = feat >= 0
    np.add.at(out, (m[ok], slot[ok], feat[ok]), add[ok])
    np.add.at(out, (m, slot, np.full_like(m, 7)), 1.0)
    return out
