"""Checkpoint / resume of a rating run (SURVEY C5, §5 "Checkpoint / resume").

The reference's only durability is the MySQL commit per batch followed by the
AMQP acks (/root/reference/worker.py:122-166,194): at-least-once delivery with
non-idempotent updates, so a crash between commit and ack double-rates a batch.
Here a run over a deterministic stream (counter-RNG windows, or a replayable
source) checkpoints

    roster state + attributes (safetensors) + {next window, stream offset,
    stream/roster specs, epoch, metrics} (JSON)

atomically (write to a temp name, fsync, rename, fsync the parent).  A crash
between the two renames of a replacement leaves only ``<name>.old``, which
``CheckpointManager.latest`` falls back to.  Resuming loads the roster and
replays from the recorded offset, so the result is bit-identical to an
uninterrupted run: exactly-once rating by construction.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Any, Dict, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file

from ..ops.rate import Roster

META = "meta.json"
TENSORS = "roster.safetensors"


def _fsync_dir(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _atomic_dir_write(final: str, writer) -> None:
    parent = os.path.dirname(os.path.abspath(final)) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=".ckpt-", dir=parent)
    writer(tmp)
    for name in os.listdir(tmp):
        with open(os.path.join(tmp, name), "rb") as f:
            os.fsync(f.fileno())
    _fsync_dir(tmp)
    if os.path.exists(final):
        old = final + ".old"
        if os.path.exists(old):
            _rmtree(old)
        os.replace(final, old)
        _fsync_dir(parent)       # from here on, a crash leaves only <final>.old
        os.replace(tmp, final)
        _fsync_dir(parent)
        _rmtree(old)
    else:
        os.replace(tmp, final)
        _fsync_dir(parent)


def _rmtree(path: str) -> None:
    for name in os.listdir(path):
        os.remove(os.path.join(path, name))
    os.rmdir(path)


def save(path: str, roster: Roster, meta: Dict[str, Any]) -> None:
    """Write one checkpoint directory (replaces an existing one atomically)."""
    tensors = {"state": roster.state.detach().cpu().contiguous(),
               "attrs": roster.attrs.detach().cpu().contiguous()}
    meta = dict(meta, epoch=roster.epoch, num_players=roster.num_players, format=1)

    def write(d):
        save_file(tensors, os.path.join(d, TENSORS))
        with open(os.path.join(d, META), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)

    _atomic_dir_write(path, write)


def load(path: str, device="cpu") -> Tuple[Roster, Dict[str, Any]]:
    t = load_file(os.path.join(path, TENSORS))
    with open(os.path.join(path, META)) as f:
        meta = json.load(f)
    # tags are only meaningful within the process that wrote them: reset on resume
    roster = Roster(t["state"].to(device), t["attrs"].to(device), epoch=None)
    return roster, meta


class CheckpointManager:
    """Keeps the latest checkpoint of a run under ``directory/latest``."""

    def __init__(self, directory: Optional[str], every: int = 1, rank: int = 0):
        self.directory = directory
        self.every = max(1, int(every))
        self.rank = rank
        self.saved = 0

    @property
    def path(self) -> Optional[str]:
        if not self.directory:
            return None
        return os.path.join(self.directory, "latest" if self.rank == 0 else "latest.r%d" % self.rank)

    def due(self, windows_done: int) -> bool:
        return bool(self.directory) and windows_done > 0 and windows_done % self.every == 0

    def maybe_save(self, windows_done: int, roster: Roster, meta: Dict[str, Any]) -> bool:
        if not self.due(windows_done):
            return False
        save(self.path, roster, dict(meta, windows_done=windows_done))
        self.saved += 1
        return True

    def latest(self, device="cpu") -> Optional[Tuple[Roster, Dict[str, Any]]]:
        """The newest complete checkpoint: ``latest``, or ``latest.old`` when a
        crash hit between the renames of a replacement."""
        p = self.path
        if not p:
            return None
        for cand in (p, p + ".old"):
            if os.path.exists(os.path.join(cand, META)) and os.path.exists(os.path.join(cand, TENSORS)):
                return load(cand, device)
        return None
