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
  dataflow launch (the fused streaming mode): each lane group folds the events
  of the match it just rated (inline, default), or aggregation waves take
  MFMA tiles (ANA_TELE_ROLE >= 0).  Inline fusion holds up to
  ANA_TELE_FUSE_MAX matches per launch -- a 500-match worker batch takes 45 us
  fused against 80 us for rating + kernel -- and above that the call runs
  ``aggregate``'s kernel after the rating instead (``BatchRater.fuses``).

Events are 8-B records (slot | type << 8 | 16-bit match tag << 16, value bits)
grouped by match with CSR offsets ``evoff[M+1]`` (layout: csrc/telemetry_core.h).  ``make_telemetry`` generates them with the
counter RNG (deterministic per global match index, device or host);
``TelemetrySource`` reads real events from an ANATEL01 file keyed by match api
id (``write_telemetry`` / ``jsonl_to_telemetry`` build one from downloaded
telemetry).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Iterable, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch

from .native import native

STAT_NAMES = ("kills", "deaths", "assists", "damage", "gold", "farm", "healing", "events")
HOST_COUNTS_MAX = 1 << 16  # make_telemetry: per-match event counts on the host up to this many matches
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


class TelemetrySource:
    """Real events for DOTELEMETRY: an ANATEL01 file (csrc/telemetry_file.cpp),
    memory-mapped and keyed by match api id (``TELEMETRY_SOURCE=<path>``).
    ``for_batch`` gathers a batch's events (pinned on a GPU) in the batch's
    match order, slots and tags -- matches without telemetry get no events."""

    def __init__(self, path: str):
        self.path = path
        self.file = native().TelemetryFile(path)

    @property
    def num_matches(self) -> int:
        return int(self.file.num_matches)

    def for_batch(self, ids: Sequence[str], K: int, device) -> Telemetry:
        device = torch.device(device)
        evoff, events = self.file.gather(list(ids), int(K), device.type == "cuda")
        return Telemetry(evoff.to(device, non_blocking=True), events.to(device, non_blocking=True))


EVENT_INDEX = {name: k for k, name in enumerate(EVENT_TYPES)}


def write_telemetry(path: str, matches: Iterable[Tuple[str, Sequence]]) -> int:
    """Write an ANATEL01 file from ``(match api id, events)`` pairs, an event
    being ``(roster, position, type, value)`` -- type an EVENT_TYPES name or
    index, value a float (ignored for kill / death / assist / other).  Returns
    the number of events."""
    ids: List[str] = []
    off = [0]
    meta: List[int] = []
    vals: List[float] = []
    for mid, evs in matches:
        ids.append(str(mid))
        for r, pos, typ, val in evs:
            t = EVENT_INDEX[typ] if isinstance(typ, str) else int(typ)
            if not (0 <= int(r) < 16 and 0 <= int(pos) < 16 and 0 <= t < 256):
                raise ValueError("event (%r, %r, %r) out of range in match %s" % (r, pos, typ, mid))
            meta.append(int(r) << 4 | int(pos) | t << 8)
            vals.append(float(val))
        off.append(len(meta))
    events = np.empty((len(meta), 2), dtype=np.int32)
    events[:, 0] = np.asarray(meta, dtype=np.int32)
    events[:, 1] = np.asarray(vals, dtype=np.float32).view(np.int32)
    native().write_telemetry_file(path, ids, torch.tensor(off, dtype=torch.int64), torch.from_numpy(events))
    return len(meta)


def jsonl_to_telemetry(src: str, dst: str) -> int:
    """Convert downloaded telemetry as JSON lines -- ``{"match": api_id,
    "events": [[roster, position, type, value], ...]}`` per line -- into an
    ANATEL01 file.  Returns the number of events."""
    def rows():
        with open(src) as f:
            for line in f:
                if line.strip():
                    d = json.loads(line)
                    yield d["match"], d.get("events", ())
    return write_telemetry(dst, rows())


def make_telemetry(spec, rec: torch.Tensor, K: int, base: int = 0,
                   ids: Optional[Sequence[str]] = None) -> Telemetry:
    """Telemetry for the matches of ``rec``: from a ``TelemetrySource`` (the
    matches' api ids ``ids``), else synthetic from a ``TelemetrySpec`` (global
    match indices base..)."""
    if isinstance(spec, TelemetrySource):
        if ids is None or len(ids) != int(rec.shape[0]):
            raise ValueError("a telemetry source needs the api id of every match")
        return spec.for_batch(ids, K, rec.device)
    M = int(rec.shape[0])
    if rec.is_cuda and M <= HOST_COUNTS_MAX:
        # a worker batch: the counts (counter RNG, same values as the device kernel) on
        # the host, so sizing the events needs no device sync -- an .item() here would
        # wait for every batch still in flight on the stream
        counts = native().gen_event_counts(M, spec.seed, spec.min_events, spec.max_events, base,
                                           torch.device("cpu"))
        off = torch.zeros(M + 1, dtype=torch.int64)
        torch.cumsum(counts, 0, out=off[1:])
        E = int(off[-1])
        evoff = off.pin_memory().to(rec.device, non_blocking=True)
    else:
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
    """fp64 numpy oracle of the aggregation.  Strict attribution, as the kernels
    and the host mirror (csrc/telemetry_core.h): an event whose 16-bit match tag
    does not name the match of its CSR range, or whose slot is >= 2K, is dropped."""
    ev = tel.events.cpu().numpy()
    M = tel.evoff.numel() - 1
    out = np.zeros((M, 2 * K, len(STAT_NAMES)), dtype=np.float64)
    if ev.shape[0] == 0:
        return out
    m = np.repeat(np.arange(M, dtype=np.int64), np.diff(tel.evoff.cpu().numpy()))  # CSR position
    slot = ev[:, 0] & 0xFF
    typ = (ev[:, 0] >> 8) & 0xFF
    tag = (ev[:, 0].astype(np.int64) >> 16) & 0xFFFF
    good = (tag == (m & 0xFFFF)) & (slot < 2 * K)
    m, slot, typ, ev = m[good], slot[good], typ[good], ev[good]
    val = ev[:, 1].view(np.float32).astype(np.float64)
    add = np.where(typ <= 2, 1.0, val)
    feat = np.where(typ <= 6, typ, -1)
    ok = feat >= 0
    np.add.at(out, (m[ok], slot[ok], feat[ok]), add[ok])
    np.add.at(out, (m, slot, np.full_like(m, 7)), 1.0)
    return out


def main(argv=None) -> int:
    """``python -m analyzer_amd.ops.telemetry convert events.jsonl out.anatel``"""
    import argparse

    ap = argparse.ArgumentParser(description="telemetry event files (ANATEL01)")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("convert", help="JSON lines -> ANATEL01")
    c.add_argument("src")
    c.add_argument("dst")
    i = sub.add_parser("info", help="matches and events of an ANATEL01 file")
    i.add_argument("path")
    a = ap.parse_args(argv)
    if a.cmd == "convert":
        print(json.dumps({"events": jsonl_to_telemetry(a.src, a.dst), "file": a.dst}))
    else:
        f = native().TelemetryFile(a.path)
        print(json.dumps({"matches": int(f.num_matches), "events": int(f.num_events)}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
