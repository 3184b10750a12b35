"""Host ingest and egress around the device pipeline.

* ``write_records`` / ``FileSource``: match records on disk (ANAREC01 files)
  are read by the native ``RecordReader`` (csrc/ingest.cpp) on a background
  thread into a ring of pinned host windows; each window is copied to the GPU on
  a dedicated copy stream (non-blocking H2D) and its pinned slot is recycled as
  soon as that copy completes -- ingest overlaps the rating of earlier windows.
* ``OutputSink``: per-window results are copied back D2H on a second copy
  stream into pinned buffers and handed to a callback once they land, so output
  egress also overlaps the next window's rating.

On the CPU the same classes run synchronously (the host mirror path).
"""
from __future__ import annotations

import collections
from typing import Callable, Deque, Iterator, Optional, Tuple

import torch

from ..ops.native import native
from ..ops.rate import RateResult


def write_records(path: str, rec: torch.Tensor, K: int) -> None:
    native().write_record_file(path, rec.detach().cpu().contiguous(), int(K))


class FileSource:
    """Iterate ``(base, rec)`` windows of a record file as device tensors."""

    def __init__(self, path: str, window: int, device="cpu", slots: int = 3):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.reader = native().RecordReader(path, int(window), int(slots), self.cuda)
        self.K = int(self.reader.K)
        self.copy_stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._inflight: Deque[Tuple[int, torch.cuda.Event]] = collections.deque()

    @property
    def num_windows(self) -> int:
        return int(self.reader.num_windows)

    def _recycle(self, block: bool) -> None:
        while self._inflight:
            slot, ev = self._inflight[0]
            if not block and not ev.query():
                return
            ev.synchronize()
            self.reader.release(slot)
            self._inflight.popleft()
            block = False

    def __iter__(self) -> Iterator[Tuple[int, torch.Tensor]]:
        while True:
            if self.cuda and len(self._inflight) >= 2:
                self._recycle(block=True)  # keep a free slot for the reader thread
            got = self.reader.acquire()
            if got is None:
                break
            slot, base, host = got
            if not self.cuda:
                rec = host.clone()
                self.reader.release(slot)
            else:
                main = torch.cuda.current_stream(self.device)
                with torch.cuda.stream(self.copy_stream):
                    rec = torch.empty(host.shape, dtype=host.dtype, device=self.device)
                    rec.copy_(host, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                main.wait_event(ev)              # consumers on the main stream see the data
                rec.record_stream(main)
                self._inflight.append((slot, ev))
                self._recycle(block=False)
            yield int(base), rec
        if self.cuda:
            while self._inflight:
                self._recycle(block=True)


class OutputSink:
    """Asynchronous D2H of per-window results into a ring of pinned host buffers.

    ``push(base, res)`` enqueues the copy of ``res`` on a copy stream behind
    everything already on the main stream and returns at once;
    ``on_ready(base, host)`` runs (on the host, from ``push``/``poll``/``flush``)
    once that copy has landed, with views into the pinned slot that stay valid
    until the callback returns.  ``copied(res)`` is the event to make the main
    stream wait on before it overwrites ``res`` (double-buffered outputs).
    Pinned slots are allocated once (``slots`` of them, grown to the largest
    window) and recycled: pinning a 2-GB window per push would cost more than
    the copy.  ``slots=0``: no ring -- every window gets fresh pinned buffers
    that the callback may keep (small windows, tests)."""

    FIELDS = ("quality", "status", "s_mu", "s_sig", "delta", "m_mu", "m_sig")

    def __init__(self, device, on_ready: Callable[[int, dict], None], slots: int = 2):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.on_ready = on_ready
        self.copy_stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.ring = int(slots) > 0
        self._slots = [None] * max(1, int(slots))
        self._next = 0
        self._pending: Deque[Tuple[int, dict, Optional[torch.cuda.Event], int, int]] = collections.deque()
        self._copied = {}
        self.bytes = 0

    def _slot(self, i: int, shape, dtype) -> torch.Tensor:
        buf = self._slots[i] if self.ring else None
        n = 1
        for d in shape:
            n *= int(d)
        if buf is None or buf.numel() < n or buf.dtype != dtype:
            buf = torch.empty(n, dtype=dtype, pin_memory=True)
            self._slots[i] = buf
        return buf[:n].view(shape)

    def push(self, base: int, res: RateResult) -> None:
        if not self.cuda:
            self.on_ready(base, {f: getattr(res, f).clone() for f in self.FIELDS})
            return
        # the ring slot we are about to reuse must have been delivered
        while self.ring and len(self._pending) >= len(self._slots):
            self.poll(block=True, limit=1)
        i = self._next
        self._next = (self._next + 1) % len(self._slots)
        main = torch.cuda.current_stream(self.device)
        done = torch.cuda.Event()
        done.record(main)
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(done)
            if res.packed is not None:  # one DMA of the packed rows, host views rebuilt
                buf = self._slot(i, res.packed.shape, torch.float32)
                buf.copy_(res.packed, non_blocking=True)
                # the caching allocator must not hand these blocks to later main-stream
                # work while this copy may still be reading them: a caller that drops
                # ``res`` right away (rate_file: a fresh result every window) is safe
                res.packed.record_stream(self.copy_stream)
                S = res.s_mu.shape[1]
                host = {"quality": buf[:, 5 * S], "status": buf.view(torch.uint8)[:, 4 * (5 * S + 1)]}
                for k, f in enumerate(("s_mu", "s_sig", "delta", "m_mu", "m_sig")):
                    host[f] = buf[:, k * S:(k + 1) * S]
                self.bytes += res.packed.numel() * 4
            else:
                host = {}
                for f in self.FIELDS:
                    src = getattr(res, f)
                    dst = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
                    dst.copy_(src, non_blocking=True)
                    src.record_stream(self.copy_stream)
                    host[f] = dst
                    self.bytes += src.numel() * src.element_size()
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        key = id(res.packed if res.packed is not None else res.s_mu)
        self._copied[key] = ev
        self._pending.append((base, host, ev, i, key))
        self.poll()

    def copied(self, res: RateResult) -> Optional[torch.cuda.Event]:
        """Event after which ``res`` may be overwritten (None: never pushed)."""
        return self._copied.get(id(res.packed if res.packed is not None else res.s_mu))

    def poll(self, block: bool = False, limit: Optional[int] = None) -> None:
        n = 0
        while self._pending and (limit is None or n < limit):
            base, host, ev, _, key = self._pending[0]
            if not block and ev is not None and not ev.query():
                return
            if ev is not None:
                ev.synchronize()
            self.on_ready(base, host)
            self._pending.popleft()
            if self._copied.get(key) is ev:  # delivered: no stale event under a recycled id
                del self._copied[key]
            n += 1

    def flush(self) -> None:
        self.poll(block=True)


def rate_file(path: str, roster, window: int, rater=None, on_result=None) -> int:
    """Rate every window of a record file in order (ingest, prepass, rating and
    egress overlapped on a GPU); ``on_result(base, host_dict)`` receives outputs."""
    from ..ops.rate import BatchRater
    from .engine import WindowPipeline

    src = FileSource(path, window, roster.device)
    pipe = WindowPipeline(rater or BatchRater(), roster, src.K)
    sink = OutputSink(roster.device, on_result, slots=0) if on_result is not None else None
    bases = []

    def windows():
        for base, rec in src:
            bases.append(base)
            yield rec

    def done(i, res):
        if sink is not None:
            sink.push(bases[i], res)

    n = pipe.run(windows(), on_result=done)
    if sink is not None:
        sink.flush()
    return n
