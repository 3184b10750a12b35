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
writes the safetensors file straight from the pinned buffer (no serialisation copy;
O_DIRECT for the block-aligned body, ``ANA_CKPT_DIRECT``), fsyncs and renames.  ``flush`` waits for every submitted checkpoint; a run is only
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
import time
from typing import Any, Dict, List, Optional, Tuple

import torch
from safetensors.torch import load_file

from ..ops.rate import Roster

META = "meta.json"
TENSORS = "roster.safetensors"
ATTRS = "attrs.safetensors"
# 1: full [P, 32] state rows (tags included); 2: base rows [P, 16] + attrs in one file;
# 3: tracks [P, 14] (the spare granule only when not NULL) + attrs in their own file
FORMAT = 3


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


# direct I/O (default): 1B matches / 10M players with a checkpoint every 8 windows 1.08-1.10 s
# against 1.34-1.47 s through the page cache (profiles/r6/rerate_attribution.log)
DIRECT_IO = os.environ.get("ANA_CKPT_DIRECT", "1") not in ("", "0", "false")
DIRECT_BLOCK = 4096

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
    # the data starts 8-B aligned; with direct I/O at a 4-KB block boundary (the JSON
    # header may carry trailing spaces, safetensors allows it)
    align = DIRECT_BLOCK if DIRECT_IO else 8
    h += b" " * (-(8 + len(h)) % align)
    head = struct.pack("<Q", len(h)) + h
    bufs = [memoryview(t.view(torch.uint8).reshape(-1).numpy()) for t in tensors.values() if t.numel()]
    if DIRECT_IO and _write_direct(path, head, bufs):
        return len(head) + off
    with open(path, "wb", buffering=0) as f:
        f.write(head)
        for mv in bufs:
            while len(mv):
                mv = mv[f.write(mv):]
    return len(head) + off


def _write_direct(path: str, head: bytes, bufs) -> bool:
    """O_DIRECT writes (ANA_CKPT_DIRECT=1): the block-aligned body of each buffer goes
    from its (page-aligned, pinned) memory straight to the device -- no page-cache copy
    and no dirty-page write-back for fsync to wait on; the unaligned tails and the header
    go through an ordinary descriptor.  False (nothing written) when the file system or
    a buffer's alignment does not allow it."""
    import mmap

    if any(b.nbytes and (b.obj.ctypes.data if hasattr(b.obj, "ctypes") else 0) % DIRECT_BLOCK for b in bufs):
        return False
    try:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_DIRECT, 0o644)
    except (OSError, AttributeError):
        return False
    tails = []
    try:
        pos = len(head)
        for mv in bufs:
            body = (len(mv) // DIRECT_BLOCK) * DIRECT_BLOCK
            o = 0
            while o < body:
                n = os.pwrite(fd, mv[o:body], pos + o)
                if n <= 0:
                    raise OSError("short direct write")
                o += n
            if body < len(mv):
                tails.append((pos + body, mv[body:]))
            pos += len(mv)
    except OSError:
        os.close(fd)
        os.remove(path)
        return False
    os.close(fd)
    fd = os.open(path, os.O_WRONLY)
    try:
        os.pwrite(fd, head, 0)
        for o, mv in tails:
            while len(mv):
                n = os.pwrite(fd, mv, o)
                o, mv = o + n, mv[n:]
    finally:
        os.close(fd)
    return True


def base_and_attrs(roster: Roster) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mu, sigma) of the 8 granules [P, 16] and the attributes [P, 4] (views on the
    roster's device; the tag words are left out)."""
    P = roster.num_players
    return roster.state.view(P, 8, 4)[:, :, 0::2].reshape(P, 16), roster.attrs


def spare_is_null(roster: Roster) -> bool:
    """Whether the spare granule 7 of every row is NULL (NaN mu and sigma), as every
    roster source writes it and nothing rates into it (csrc/common.h): then format 3
    leaves it out -- 56 instead of 64 B of ratings per player (syncs once)."""
    P = roster.num_players
    return bool(torch.isnan(roster.state.view(P, 8, 4)[:, 7, 0::2]).all())


def _state_from_base(base: torch.Tensor) -> torch.Tensor:
    P = base.shape[0]
    state = torch.zeros((P, 32), dtype=torch.float32, device=base.device)
    state.view(P, 8, 4)[:, :, 0::2] = base.view(P, 8, 2)
    return state


def _meta(roster: Roster, meta: Dict[str, Any], spare: bool) -> Dict[str, Any]:
    return dict(meta, epoch=roster.epoch, num_players=roster.num_players, format=FORMAT, spare_saved=spare)


def _write(path: str, tracks: torch.Tensor, attrs: Optional[torch.Tensor], meta: Dict[str, Any],
           fsync: bool = True, link_attrs: Optional[str] = None) -> None:
    """One checkpoint directory: ``tracks`` [P, 14] (or [P, 16] with the spare granule),
    ``attrs`` [P, 4] -- written, or hard-linked from ``link_attrs`` (an unchanged attrs
    file of the previous checkpoint: no bytes written)."""
    def write(d):
        write_safetensors(os.path.join(d, TENSORS), {"tracks": tracks})
        dst = os.path.join(d, ATTRS)
        linked = False
        if link_attrs is not None and os.path.exists(link_attrs):
            try:
                os.link(link_attrs, dst)
                linked = True
            except OSError:  # another file system: write them
                linked = False
        if not linked:
            write_safetensors(dst, {"attrs": attrs})
        with open(os.path.join(d, META), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)

    _atomic_dir_write(path, write, fsync)


def _tracks(base: torch.Tensor, spare: bool) -> torch.Tensor:
    return base if spare else base[:, :14]


def save(path: str, roster: Roster, meta: Dict[str, Any], fsync: bool = True) -> None:
    """Write one checkpoint directory synchronously (replaces an existing one atomically)."""
    base, attrs = base_and_attrs(roster)
    spare = not spare_is_null(roster)
    _write(path, _tracks(base, spare).detach().cpu().contiguous(), attrs.detach().cpu().contiguous(),
           _meta(roster, meta, spare), fsync)


def load(path: str, device="cpu") -> Tuple[Roster, Dict[str, Any]]:
    """Formats 1 (full rows), 2 (base rows + attrs in one file) and 3 (tracks; attrs in
    their own file, hard-linked between checkpoints while unchanged)."""
    t = load_file(os.path.join(path, TENSORS))
    with open(os.path.join(path, META)) as f:
        meta = json.load(f)
    # tags are only meaningful within the process that wrote them: reset on resume
    if "state" in t:      # format 1
        state = t["state"].clone()
        state.view(-1, 8, 4)[:, :, 1::2] = 0.0
    elif "base" in t:     # format 2
        state = _state_from_base(t["base"])
    else:                 # format 3
        tr = t["tracks"]
        base = torch.full((tr.shape[0], 16), float("nan"), dtype=torch.float32)
        base[:, :tr.shape[1]] = tr
        state = _state_from_base(base)
    attrs = t["attrs"] if "attrs" in t else load_file(os.path.join(path, ATTRS))["attrs"]
    roster = Roster(state.to(device), attrs.to(device), epoch=None)
    return roster, meta


class AsyncCheckpointer:
    """Checkpoints written beside the rating (module docstring).  ``submit`` is
    stream-ordered on the caller's current stream: it snapshots the roster as the
    work enqueued so far leaves it, and returns without waiting for the GPU.

    ``static_attrs``: the caller guarantees the attributes never change during the run
    (runtime/rerate.py: the kernels only read them, csrc/dataflow.hip) -- they are copied
    to the host once, written with the first checkpoint and hard-linked into the later ones."""

    def __init__(self, device, num_players: int, buffers: int = 2, fsync: bool = True,
                 static_attrs: bool = False):
        self.device = torch.device(device)
        self.P = int(num_players)
        self.fsync = bool(fsync)
        self.static_attrs = bool(static_attrs)
        self.cuda = self.device.type == "cuda"
        self.spare: Optional[bool] = None  # spare granule saved (decided at the first submit)
        f = dict(dtype=torch.float32)
        self._f = f
        self._stage = None
        self._staged: Optional[torch.cuda.Event] = None     # staging free again (its D2H done)
        self._host: List[Tuple[torch.Tensor, Optional[torch.Tensor]]] = []
        self._nbuf = max(1, buffers)
        self._attrs_host: Optional[torch.Tensor] = None    # static attrs, copied once
        self._attrs_file: Optional[str] = None             # their last committed file
        self._copy = torch.cuda.Stream(self.device) if self.cuda else None
        self._next = 0
        # one writer thread, FIFO: checkpoints commit in submission order (two writers
        # would race on the renames, and an older snapshot could land last)
        self._queue: "queue.Queue" = queue.Queue()
        self._free = [threading.Event() for _ in range(self._nbuf)]  # buffer i may be refilled
        for e in self._free:
            e.set()
        self._errors: List[BaseException] = []
        self._writer: Optional[threading.Thread] = None
        self.written = 0
        self.bytes = 0
        self.write_s: List[float] = []  # seconds per committed checkpoint (write + fsync + rename)
        self.flush_s = 0.0              # seconds the callers waited in flush()

    def _buffers(self, roster: Roster) -> None:
        if self._host:
            return
        self.spare = not spare_is_null(roster)
        w = 16 if self.spare else 14
        f, pin = self._f, self.cuda
        keep_attrs = not self.static_attrs
        if self.cuda:
            self._stage = (torch.empty((self.P, w), device=self.device, **f),
                           torch.empty((self.P, 4), device=self.device, **f) if keep_attrs else None)
        self._host = [(torch.empty((self.P, w), pin_memory=pin, **f),
                       torch.empty((self.P, 4), pin_memory=pin, **f) if keep_attrs else None)
                      for _ in range(self._nbuf)]

    def _run(self) -> None:
        while True:
            item = self._queue.get()
            if item is None:
                return
            i, path, meta, done, attrs = item
            hb, _ = self._host[i]
            try:
                if done is not None:
                    done.synchronize()
                link = self._attrs_file if self.static_attrs else None
                t0 = time.perf_counter()
                _write(path, hb, attrs, meta, self.fsync, link_attrs=link)
                self.write_s.append(time.perf_counter() - t0)
                if self.static_attrs:
                    self._attrs_file = os.path.join(path, ATTRS)
                self.written += 1
                self.bytes += hb.numel() * 4 + (0 if link else attrs.numel() * 4)
            except BaseException as e:  # re-raised by the next submit / flush
                self._errors.append(e)
            finally:
                self._free[i].set()
                self._queue.task_done()

    def prepare(self, roster: Roster) -> None:
        """Allocate the staging and pinned host buffers (and, with static attributes, take
        their one host copy) now -- a run calls it before its first window, so page-locking
        ~1 GB of host memory does not land inside the run's first checkpoint."""
        self._buffers(roster)
        if self.static_attrs and self._attrs_host is None:
            self._attrs_host = roster.attrs.detach().to("cpu", copy=True).contiguous()

    def submit(self, path: str, roster: Roster, meta: Dict[str, Any]) -> None:
        self._buffers(roster)
        i = self._next
        self._next = (self._next + 1) % self._nbuf
        self._free[i].wait()  # back-pressure: that buffer's write is still running
        self._raise()
        self._free[i].clear()
        hb, ha = self._host[i]
        base, attrs = base_and_attrs(roster)
        tracks = _tracks(base, self.spare)
        done = None
        if self.static_attrs and self._attrs_host is None:
            self._attrs_host = attrs.detach().to("cpu", copy=True).contiguous()  # once (syncs)
        if self.cuda:
            main = torch.cuda.current_stream(self.device)
            if self._staged is not None:
                main.wait_event(self._staged)  # the previous snapshot left the staging buffer
            sb, sa = self._stage
            sb.copy_(tracks)
            if sa is not None:
                sa.copy_(attrs)
            snap = torch.cuda.Event()
            snap.record(main)
            self._copy.wait_event(snap)
            with torch.cuda.stream(self._copy):
                hb.copy_(sb, non_blocking=True)
                if sa is not None:
                    ha.copy_(sa, non_blocking=True)
                done = torch.cuda.Event()
                done.record(self._copy)
            self._staged = done
        else:
            hb.copy_(tracks)
            if ha is not None:
                ha.copy_(attrs)
        if self._writer is None:
            self._writer = threading.Thread(target=self._run, name="checkpoint-writer", daemon=True)
            self._writer.start()
        self._queue.put((i, path, _meta(roster, meta, self.spare), done,
                         self._attrs_host if self.static_attrs else ha))

    def flush(self) -> None:
        """Wait until every submitted checkpoint is committed (renamed into place)."""
        t0 = time.perf_counter()
        self._queue.join()
        self.flush_s += time.perf_counter() - t0
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

    def __init__(self, directory: Optional[str], every: int = 1, rank: int = 0, static_attrs: bool = False):
        self.directory = directory
        self.static_attrs = bool(static_attrs)
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

    def _use_async(self, roster: Roster) -> bool:
        return roster.state.device.type == "cuda" and \
            os.environ.get("ANA_CKPT_ASYNC", "1") not in ("", "0", "false")

    def prepare(self, roster: Roster) -> None:
        """Set up the asynchronous writer's buffers ahead of the first save (no-op without a
        directory or on the host path)."""
        if not self.directory or not self._use_async(roster):
            return
        if self._async is None:
            self._async = AsyncCheckpointer(roster.state.device, roster.num_players, fsync=self.fsync,
                                            static_attrs=self.static_attrs)
        self._async.prepare(roster)

    def maybe_save(self, windows_done: int, roster: Roster, meta: Dict[str, Any]) -> bool:
        if not self.due(windows_done):
            return False
        meta = dict(meta, windows_done=windows_done)
        if self._use_async(roster):
            if self._async is None:
                self._async = AsyncCheckpointer(roster.state.device, roster.num_players, fsync=self.fsync,
                                                static_attrs=self.static_attrs)
            self._async.submit(self.path, roster, meta)
        else:
            save(self.path, roster, meta, self.fsync)
        self.saved += 1
        return True

    def flush(self) -> None:
        if self._async is not None:
            self._async.flush()

    def stats(self) -> Dict[str, float]:
        """Asynchronous writer timing: checkpoints committed, mean / max seconds per commit
        and the seconds callers waited in flush() (empty without the writer)."""
        a = self._async
        if a is None or not a.write_s:
            return {}
        return {"checkpoints": float(len(a.write_s)), "write_s_mean": sum(a.write_s) / len(a.write_s),
                "write_s_max": max(a.write_s), "flush_wait_s": a.flush_s}

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
