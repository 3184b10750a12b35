"""Tracing (SURVEY §5 "Tracing / profiling"; the reference has none).

``trace_range(name)`` marks a host-side region:

* with ``ANA_TRACE=1`` it is recorded by an in-process tracer (monotonic
  timestamps, thread id) that ``dump_chrome_trace(path)`` writes as Chrome
  trace-event JSON (chrome://tracing, Perfetto);
* on a ROCm device it also pushes a ROCTX range (``torch.cuda.nvtx`` maps to
  roctx on ROCm builds), so ``rocprofv3 --marker-trace --kernel-trace`` shows
  the engine's phases (schedule, rate, merge, checkpoint) around the kernels.

Disabled (the default) it costs one dict lookup.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from typing import Dict, List

_events: List[Dict] = []
_lock = threading.Lock()


def enabled() -> bool:
    """``EngineConfig.trace`` (ANA_TRACE), read without building the whole config:
    this runs around every traced region."""
    v = os.environ.get("ANA_TRACE")
    return bool(v) and v != "0"


def _roctx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover - torch without nvtx/roctx
        return None
    return None


@contextlib.contextmanager
def trace_range(name: str, **args):
    if not enabled():
        yield
        return
    rx = _roctx()
    if rx is not None:
        try:
            rx.range_push(name)
        except Exception:  # roctx unavailable in this build: host timing only
            rx = None
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        t1 = time.perf_counter_ns()
        if rx is not None:
            rx.range_pop()
        with _lock:
            _events.append({"name": name, "ph": "X", "ts": t0 / 1000.0, "dur": (t1 - t0) / 1000.0,
                            "pid": os.getpid(), "tid": threading.get_ident() % (1 << 31),
                            "args": args})


def events() -> List[Dict]:
    with _lock:
        return list(_events)


def clear() -> None:
    with _lock:
        _events.clear()


def dump_chrome_trace(path: str) -> int:
    ev = events()
    with open(path, "w") as f:
        json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
    return len(ev)
