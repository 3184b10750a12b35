"""Checkpoint / resume of a rating run (SURVEY C5, §5 "Checkpoint / resume").

The reference's only durability is the MySQL commit per batch followed by the
AMQP acks (/root/reference/worker.py:122-166,194): at-least-once delivery with
non-idempotent updates, so a crash between commit and ack double-rates a batch.
Here a run over a deterministic stream (counter-RNG windows, or a replayable
source) checkpoints

    the roster's (mu, sigma) of every track + attributes (safetensors: ``base``
    [P, 16] and ``attrs`` [P, 4] fp32, 80 B per player) + {next window, stream
    offset, stream/roster specs, metrics} (JSON)

atomically (write to a temp name, fsync, rename, fsync the parent).  A crash
between the two renames of a replacement leaves only ``<name>.old``, which
``CheckpointManager.latest`` falls back to.  Resuming loads the roster and
replays from the recorded offset, so the result is bit-identical to an
uninterrupted run: exactly-once rating by construction.  The dataflow tags of a
row (csrc/common.h) are per-process and are not saved: a resumed roster starts
with zero tags, as ``load`` always did.

**Asynchronous writes** (``AsyncCheckpointer``, the default of runtime/rerate.py on
a GPU).  A synchronous save of a 10M-player roster stalls the window pipeline for
~0.56 s (D2H of 1.4 GB pageable, serialisation, write, fsync: profiles/r6/
rerate_attribution.log).  Instead the rating stream only gathers the 80-B rows into
a device staging buffer (~0.3 ms for 10M players); a copy stream moves them into
one of two pinned host buffers beside the next windows' rating, and a writer thread
writes the safetensors file straight from the pinned buffer (no serialisation copy),
fsyncs and renames.  ``flush`` waits for every submitted checkpoint; a run is only
reported finished once its last checkpoint is committed.  When both host buffers are
still being written, the next ``submit`` waits (back-pressure, never a dropped
checkpoint).
"""
from __future__ import annotations

import json
import os
import queue
import struct
import tempfile
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional, Tuple

import torch
from safetensors.torch import load_file

from ..ops.rate import Roster

META = "meta.json"
TENSORS = "roster.safetensors"
FORMAT = 2  # 1: full [P, 32] state rows (tags included); 2: base rows [P, 16] + attrs


def _fsync_dir(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _atomic_dir_write(final: str, writer, fsync: bool = True) -> None:
    parent = os.path.dirname(os.path.abspath(final)) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=".ckpt-", dir=parent)
    writer(tmp)
    if fsync:
        for name in os.listdir(tmp):
            with open(os.path.join(tmp, name), "rb") as f:
                os.fsync(f.fileno())
        _fsync_dir(tmp)
    if os.path.exists(final):
        old = final + ".old"
        if os.path.exists(old):
            _rmtree(old)
        os.replace(final, old)
        if fsync:
            _fsync_dir(parent)   # from here on, a crash leaves only <final>.old
        os.replace(tmp, final)
        if fsync:
            _fsync_dir(parent)
        _rmtree(old)
    else:
        os.replace(tmp, final)
        if fsync:
            _fsync_dir(parent)


def _rmtree(path: str) -> None:
    for name in os.listdir(path):
        os.remove(os.path.join(path, name))
    os.rmdir(path)


WRITE_PIECE = 64 << 20
WRITE_THREADS = int(os.environ.get("ANA_CKPT_WRITE_THREADS") or 8)

_ST_DTYPES = {torch.float32: "F32", torch.float64: "F64", torch.int32: "I32", torch.int64: "I64",
              torch.uint8: "U8"}


def write_safetensors(path: str, tensors: Dict[str, torch.Tensor], metadata: Optional[Dict[str, str]] = None) -> int:
    """Write contiguous CPU tensors as one safetensors file, straight from their
    memory (header, then each tensor's bytes; no serialisation copy -- the pinned
    staging buffers of ``AsyncCheckpointer`` go to the file as they are).  Readable
    by ``safetensors.torch.load_file``.  Returns the bytes written."""
    header: Dict[str, Any] = {}
    off = 0
    for name, t in tensors.items():
        if t.device.type != "cpu" or not t.is_contiguous():
            raise ValueError("write_safetensors: %s must be a contiguous CPU tensor" % name)
        n = t.numel() * t.element_size()
        header[name] = {"dtype": _ST_DTYPES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        off += n
    if metadata:
        header["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    h = json.dumps(header, separators=(",", ":")).encode()
    h += b" " * (-len(h) % 8)  # the data starts 8-B aligned
    head = struct.pack("<Q", len(h)) + h
    # the payload goes to the file in 64-MB pieces from WRITE_THREADS threads (pwrite at
    # their offsets; the copies into the page cache run in parallel, the GIL is released
    # in the syscall): one thread writes ~3.5 GB/s on the GPU box (profiles/r6/
    # rerate_attribution.log), the checkpoint of a 10M-player roster is 800 MB
    pieces = []
    pos = len(head)
    for t in tensors.values():
        if t.numel():
            mv = memoryview(t.view(torch.uint8).reshape(-1).numpy())
            for a in range(0, len(mv), WRITE_PIECE):
                pieces.append((pos + a, mv[a:a + WRITE_PIECE]))
        pos += t.numel() * t.element_size()
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        os.pwrite(fd, head, 0)

        def put(item):
            o, mv = item
            while len(mv):
                n = os.pwrite(fd, mv, o)
                o, mv = o + n, mv[n:]

        if len(pieces) > 1 and WRITE_THREADS > 1:
            with ThreadPoolExecutor(WRITE_THREADS) as ex:
                list(ex.map(put, pieces))
        else:
            for it in pieces:
                put(it)
    finally:
        os.close(fd)
    return len(head) + off


def base_and_attrs(roster: Roster) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mu, sigma) of the 8 granules [P, 16] and the attributes [P, 4] (views on the
    roster's device; the tag words are left out)."""
    P = roster.num_players
    return roster.state.view(P, 8, 4)[:, :, 0::2].reshape(P, 16), roster.attrs


def _state_from_base(base: torch.Tensor) -> torch.Tensor:
    P = base.shape[0]
    state = torch.zeros((P, 32), dtype=torch.float32, device=base.device)
    state.view(P, 8, 4)[:, :, 0::2] = base.view(P, 8, 2)
    return state


def _meta(roster: Roster, meta: Dict[str, Any]) -> Dict[str, Any]:
    return dict(meta, epoch=roster.epoch, num_players=roster.num_players, format=FORMAT)


def _write(path: str, base: torch.Tensor, attrs: torch.Tensor, meta: Dict[str, Any], fsync: bool = True) -> None:
    def write(d):
        write_safetensors(os.path.join(d, TENSORS), {"base": base, "attrs": attrs})
        with open(os.path.join(d, META), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)

    _atomic_dir_write(path, write, fsync)


def save(path: str, roster: Roster, meta: Dict[str, Any], fsync: bool = True) -> None:
    """Write one checkpoint directory synchronously (replaces an existing one atomically)."""
    base, attrs = base_and_attrs(roster)
    _write(path, base.detach().cpu().contiguous(), attrs.detach().cpu().contiguous(), _meta(roster, meta), fsync)


def load(path: str, device="cpu") -> Tuple[Roster, Dict[str, Any]]:
    t = load_file(os.path.join(path, TENSORS))
    with open(os.path.join(path, META)) as f:
        meta = json.load(f)
    # tags are only meaningful within the process that wrote them: reset on resume
    state = t["state"] if "state" in t else _state_from_base(t["base"])  # format 1 / 2
    if "state" in t:
        state = state.clone()
        state.view(-1, 8, 4)[:, :, 1::2] = 0.0
    roster = Roster(state.to(device), t["attrs"].to(device), epoch=None)
    return roster, meta


class AsyncCheckpointer:
    """Checkpoints written beside the rating (module docstring).  ``submit`` is
    stream-ordered on the caller's current stream: it snapshots the roster as the
    work enqueued so far leaves it, and returns without waiting for the GPU."""

    def __init__(self, device, num_players: int, buffers: int = 2, fsync: bool = True):
        self.device = torch.device(device)
        self.P = int(num_players)
        self.fsync = bool(fsync)
        self.cuda = self.device.type == "cuda"
        f = dict(dtype=torch.float32)
        # device staging (the copy stream reads it while the rating goes on)
        self._stage = ((torch.empty((self.P, 16), device=self.device, **f),
                        torch.empty((self.P, 4), device=self.device, **f)) if self.cuda else None)
        self._staged: Optional[torch.cuda.Event] = None     # staging free again (its D2H done)
        self._host = [(torch.empty((self.P, 16), pin_memory=self.cuda, **f),
                       torch.empty((self.P, 4), pin_memory=self.cuda, **f)) for _ in range(max(1, buffers))]
        self._copy = torch.cuda.Stream(self.device) if self.cuda else None
        self._next = 0
        # one writer thread, FIFO: checkpoints commit in submission order (two writers
        # would race on the renames, and an older snapshot could land last)
        self._queue: "queue.Queue" = queue.Queue()
        self._free = [threading.Event() for _ in self._host]  # buffer i may be refilled
        for e in self._free:
            e.set()
        self._errors: List[BaseException] = []
        self._writer: Optional[threading.Thread] = None
        self.written = 0
        self.bytes = 0

    def _run(self) -> None:
        while True:
            item = self._queue.get()
            if item is None:
                return
            i, path, meta, done = item
            hb, ha = self._host[i]
            try:
                if done is not None:
                    done.synchronize()
                _write(path, hb, ha, meta, self.fsync)
                self.written += 1
                self.bytes += (hb.numel() + ha.numel()) * 4
            except BaseException as e:  # re-raised by the next submit / flush
                self._errors.append(e)
            finally:
                self._free[i].set()
                self._queue.task_done()

    def submit(self, path: str, roster: Roster, meta: Dict[str, Any]) -> None:
        i = self._next
        self._next = (self._next + 1) % len(self._host)
        self._free[i].wait()  # back-pressure: that buffer's write is still running
        self._raise()
        self._free[i].clear()
        hb, ha = self._host[i]
        base, attrs = base_and_attrs(roster)
        done = None
        if self.cuda:
            main = torch.cuda.current_stream(self.device)
            if self._staged is not None:
                main.wait_event(self._staged)  # the previous snapshot left the staging buffer
            sb, sa = self._stage
            sb.copy_(base)
            sa.copy_(attrs)
            snap = torch.cuda.Event()
            snap.record(main)
            self._copy.wait_event(snap)
            with torch.cuda.stream(self._copy):
                hb.copy_(sb, non_blocking=True)
                ha.copy_(sa, non_blocking=True)
                done = torch.cuda.Event()
                done.record(self._copy)
            self._staged = done
        else:
            hb.copy_(base)
            ha.copy_(attrs)
        if self._writer is None:
            self._writer = threading.Thread(target=self._run, name="checkpoint-writer", daemon=True)
            self._writer.start()
        self._queue.put((i, path, _meta(roster, meta), done))

    def flush(self) -> None:
        """Wait until every submitted checkpoint is committed (renamed into place)."""
        self._queue.join()
        self._raise()

    def close(self) -> None:
        self.flush()
        if self._writer is not None:
            self._queue.put(None)
            self._writer.join()
            self._writer = None

    def _raise(self) -> None:
        if self._errors:
            e = self._errors.pop(0)
            raise RuntimeError("asynchronous checkpoint write failed: %s" % e) from e


class CheckpointManager:
    """Keeps the latest checkpoint of a run under ``directory/latest``.

    ``asynchronous``: writes go through an ``AsyncCheckpointer`` (default on a GPU
    device, ``ANA_CKPT_ASYNC=0`` turns it off); ``flush`` commits what is in flight."""

    def __init__(self, directory: Optional[str], every: int = 1, rank: int = 0):
        self.directory = directory
        self.every = max(1, int(every))
        self.rank = rank
        self.saved = 0
        self.fsync = os.environ.get("ANA_CKPT_FSYNC", "1") not in ("", "0", "false")
        self._async: Optional[AsyncCheckpointer] = None

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
        meta = dict(meta, windows_done=windows_done)
        use_async = roster.state.device.type == "cuda" and \
            os.environ.get("ANA_CKPT_ASYNC", "1") not in ("", "0", "false")
        if use_async:
            if self._async is None:
                self._async = AsyncCheckpointer(roster.state.device, roster.num_players, fsync=self.fsync)
            self._async.submit(self.path, roster, meta)
        else:
            save(self.path, roster, meta, self.fsync)
        self.saved += 1
        return True

    def flush(self) -> None:
        if self._async is not None:
            self._async.flush()

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
