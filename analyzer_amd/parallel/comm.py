"""Process-group plumbing and small collectives.

One process per GPU, ``torch.distributed`` with backend ``nccl`` (RCCL on ROCm,
over xGMI) for device tensors and ``gloo`` for the CPU tests.  The reference has
no collectives at all: its replicas share state through MySQL rows and
messages through RabbitMQ (/root/reference/worker.py:44-46,85-92).

* ``init_from_env``  -- RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (torchrun).
* ``broadcast_roster`` (C3) -- the initial replicated roster from one rank.
* ``reduce_counts`` (C4) -- status counters and timings summed / maxed over ranks.
* ``shard`` -- contiguous block partition of a range (time-axis sharding, P1/P4).
* ``exclusive_scan`` (C1') -- per-row prefix sum over ranks (causal re-sweeps of
  parallel/sweep.py) as two all-to-alls.
* ``SplitExchange`` (C1 + C1') -- the merge's collective since round 6: all-to-all ->
  owner reduce -> all-gather of the sums on the critical path (an all-reduce's volume),
  the prefixes' return all-to-all deferred beside the next window's rating.
* ``scan_and_sum`` (C1 + C1') -- the round-5 collective when records are corrected:
  the sum over ranks AND each rank's exclusive prefix from one exchange (two
  all-to-alls + an all-gather of the block sums: 3 (N-1)/N of the buffer per rank,
  against 2 (N-1)/N for the all-reduce alone and 4 (N-1)/N for both separately).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist


def world(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _staged(t: torch.Tensor, group=None) -> bool:
    """gloo moves host memory only: device tensors are staged through the host
    (the 1-GPU multi-rank rehearsal; RCCL takes device tensors directly)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_to_all_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """``all_to_all_single`` over equal row blocks (one per rank)."""
    if _staged(inp, group):
        o = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=group)


def exclusive_scan(t: torch.Tensor, group=None) -> torch.Tensor:
    """Row-wise exclusive prefix sum over ranks: rank r gets sum_{q<r} t_q
    (zeros on rank 0), summed in rank order.

    Two all-to-alls instead of a chain: rank b owns row block b, receives block b
    of every rank, prefix-sums it in rank order and sends each rank its prefix
    back.  Each rank moves 2(N-1)/N of the buffer -- an all-reduce's volume --
    and on xGMI's full mesh every block travels its own point-to-point link, so
    the scan costs about one all-reduce rather than log2(N) dependent hops."""
    _, size = world(group)
    if size <= 1:
        return torch.zeros_like(t)
    P = t.shape[0]
    C = t[0].numel() if P else 1
    blk = -(-P // size)
    send = t.new_zeros((size * blk, C))
    send[:P] = t.reshape(P, C)
    recv = torch.empty_like(send)
    all_to_all_rows(recv, send, group)  # recv block q = rank q's rows of my block
    r3 = recv.view(size, blk, C)
    ex = torch.zeros_like(r3)
    if size > 1:
        torch.cumsum(r3[:-1], 0, out=ex[1:])
    back = torch.empty_like(send)
    all_to_all_rows(back, ex.view(size * blk, C), group)  # block b = my prefix of block b
    return back[:P].view_as(t)


def all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """``all_gather_into_tensor`` of equal row blocks (gloo + device: staged)."""
    if _staged(inp, group):
        o = torch.empty_like(out, device="cpu")
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def scan_and_sum(t: torch.Tensor, group=None, force: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """(exclusive prefix over ranks, sum over ranks) of ``t``, row-wise.  Rank b
    owns row block b: one all-to-all brings it block b of every rank, which it
    prefix-sums and sums in rank order (floating types in fp32, rounded once to the
    wire type); a second all-to-all returns each rank its prefix, an all-gather the
    block sums.  One rank: (zeros, t) -- through the exchanges anyway with ``force`` (tests
    of the collective path on a one-rank communicator)."""
    _, size = world(group)
    if size <= 1 and not force:
        return torch.zeros_like(t), t
    P = t.shape[0]
    C = t[0].numel() if P else 1
    blk = -(-P // size)
    send = t.new_zeros((size * blk, C))
    send[:P] = t.reshape(P, C)
    recv = torch.empty_like(send)
    all_to_all_rows(recv, send, group)  # recv block q = rank q's rows of my block
    r3 = recv.view(size, blk, C)
    acc = r3.float() if t.is_floating_point() else r3
    cs = torch.cumsum(acc, 0)
    ex = torch.zeros_like(cs)
    ex[1:] = cs[:-1]
    back = torch.empty_like(send)
    all_to_all_rows(back, ex.to(t.dtype).view(size * blk, C), group)  # block b = my prefix of block b
    total = torch.empty_like(send)
    all_gather_rows(total, cs[-1].to(t.dtype).contiguous(), group)
    return back[:P].view_as(t), total[:P].view_as(t)


def _row_bytes(x: torch.Tensor, P: int) -> torch.Tensor:
    return x.reshape(P, -1).contiguous().view(torch.uint8)


def scan_and_sum_rows(t: torch.Tensor, extra: torch.Tensor, group=None, force: bool = False):
    """``scan_and_sum`` of ``t`` whose exchanges also carry ``extra`` (rows summed,
    not scanned) in the same payload: (prefix of t, total of t, total of extra) from
    one all-to-all, one all-to-all back and one all-gather -- the DP merge's messages
    and touch counts without a separate all-reduce (a collective launch per merge).
    The rows travel as bytes and are read back through typed views.  ``force``: as
    scan_and_sum."""
    _, size = world(group)
    if size <= 1 and not force:
        return torch.zeros_like(t), t, extra
    P = t.shape[0]
    bt, be = _row_bytes(t, P), _row_bytes(extra, P)
    ct, C = bt.shape[1], bt.shape[1] + be.shape[1]
    if C % t.element_size() or C % extra.element_size() or ct % extra.element_size():
        p, s = scan_and_sum(t, group, force)  # rows that do not view back: two exchanges
        all_reduce_sum(extra, group)
        return p, s, extra
    blk = -(-P // size)
    send = torch.zeros((size * blk, C), dtype=torch.uint8, device=t.device)
    send[:P, :ct] = bt
    send[:P, ct:] = be
    recv = torch.empty_like(send)
    all_to_all_rows(recv, send, group)  # recv block q = rank q's rows of my block
    r3 = recv.view(size, blk, C)
    tv = r3[..., :ct].view(t.dtype)
    ev = r3[..., ct:].view(extra.dtype)
    cs = torch.cumsum(tv.float() if t.is_floating_point() else tv, 0)
    ex = torch.zeros_like(cs)
    ex[1:] = cs[:-1]
    back = torch.empty((size * blk, ct), dtype=torch.uint8, device=t.device)
    all_to_all_rows(back, ex.to(t.dtype).reshape(size * blk, -1).view(torch.uint8), group)
    tot = torch.empty((blk, C), dtype=torch.uint8, device=t.device)
    tot[:, :ct] = cs[-1].to(t.dtype).contiguous().view(torch.uint8)
    tot[:, ct:] = ev.sum(0).to(extra.dtype).contiguous().view(torch.uint8)
    total = torch.empty((size * blk, C), dtype=torch.uint8, device=t.device)
    all_gather_rows(total, tot, group)
    prefix = back[:P].view(t.dtype).view_as(t)
    return (prefix, total[:P, :ct].contiguous().view(t.dtype).view_as(t),
            total[:P, ct:].contiguous().view(extra.dtype).view_as(extra))


def scan_and_sum_start(t: torch.Tensor, group=None, stream=None, extra: Optional[torch.Tensor] = None,
                       force: bool = False):
    """``scan_and_sum`` in flight: returns ``finish() -> (prefix, total)``.  With RCCL
    and a side ``stream`` the two all-to-alls, the block scan between them, the
    all-gather -- which also carry ``extra``, summed in place (scan_and_sum_rows) --
    all run on that stream,
    which first waits for the current one; ``finish`` makes the current stream wait
    for it -- the caller's stream stays free for other work in between (the DP merge
    corrects the previous window's records there).  gloo / one rank / no stream:
    done at once, ``finish`` only returns it."""
    _, size = world(group)

    def run():
        if extra is None:
            return scan_and_sum(t, group, force)
        p, s, e = scan_and_sum_rows(t, extra, group, force)
        if e is not extra:
            extra.copy_(e)
        return p, s
    side = stream is not None and t.is_cuda and (size > 1 or force) and not _staged(t, group)
    if not side:
        res = run()
        return lambda: res
    cur = torch.cuda.current_stream(t.device)
    stream.wait_stream(cur)
    with torch.cuda.stream(stream):
        res = run()
    done = torch.cuda.Event()
    done.record(stream)

    def finish():
        now = torch.cuda.current_stream(t.device)
        now.wait_event(done)
        for x in res:
            if x is not t:  # allocated on the side stream, read on this one
                x.record_stream(now)
        return res
    return finish


def block_reduce_rows(recv: torch.Tensor, n: int, dtype: torch.dtype, want_prefix: bool):
    """The owner reduce of the split exchange on the host (csrc/sweep.hip
    sweep_block_reduce_kernel, bit for bit): recv [n * blk, 8] int32 words -- 7 words of
    two ``dtype`` halves (the messages) and the touch word -- -> (total [blk, 8],
    exclusive prefixes [n * blk, 7] or None).  Halves are summed in fp32 in rank order and
    rounded once; the touch words are summed as integers."""
    blk = recv.shape[0] // n
    r = recv.view(n, blk, 8)
    halves = r[..., :7].contiguous().view(dtype)  # [n, blk, 14]
    acc = torch.zeros((blk, 14), dtype=torch.float32, device=recv.device)
    pref = torch.empty((n, blk, 7), dtype=torch.int32, device=recv.device) if want_prefix else None
    for q in range(n):
        if pref is not None:
            pref[q] = acc.to(dtype).view(torch.int32)
        acc = acc + halves[q].float()
    total = torch.empty((blk, 8), dtype=torch.int32, device=recv.device)
    total[:, :7] = acc.to(dtype).view(torch.int32)
    total[:, 7] = r[..., 7].sum(0, dtype=torch.int64).to(torch.int32)
    return total, (pref.view(n * blk, 7) if pref is not None else None)


class SplitExchange:
    """The DP merge's collective, split at what the next window needs (SURVEY C1;
    parallel/sweep.py ``merge_split``).

    Every rank holds operand rows op [P, 8] int32 words (7 words of two bf16 / fp16
    message halves + the packed touch word).  The next window's roster needs only the
    SUM over ranks; only this window's records need each rank's exclusive PREFIX.  So:

    * critical (``total``): all-to-all (rank b receives row block b of every rank) ->
      owner reduce (csrc/sweep.hip sweep_block_reduce: the block's sum AND every rank's
      prefix of it, one pass) -> all-gather of the block sums.  2 (N-1)/N of the buffer
      per rank: an all-reduce's volume, where the round-5 scan moved 3 (N-1)/N before
      the decode could start.
    * deferred (``prefix``): the all-to-all that returns each rank its prefix of every
      block, (N-1)/N of 7/8 of the buffer, enqueued right behind the critical part on the
      collective stream -- it runs beside the decode and the next window's rating, and
      only the record correction (off the critical path too) waits for it.

    On xGMI's point-to-point mesh every block of an all-to-all travels its own link, so
    the split costs about one all-reduce on the critical path.  ``stream``: the
    collective stream (RCCL); gloo / host tensors run synchronously (the host reduce is
    ``block_reduce_rows``, bit-identical to the kernel).  ``force``: run the exchanges on
    a one-rank group (tests)."""

    def __init__(self, op: torch.Tensor, dtype: torch.dtype, group=None, stream=None,
                 want_prefix: bool = True, force: bool = False):
        _, size = world(group)
        self.P = int(op.shape[0])
        self.size = size
        self.dtype = dtype
        self._prefix = None
        self._pref = None
        self._total = None
        self._ev_total = self._ev_prefix = None
        run_side = stream is not None and op.is_cuda and not _staged(op, group)
        blk = -(-self.P // size) if size > 0 else self.P
        if blk * size == self.P:
            send = op
        else:
            send = op.new_zeros((size * blk, 8))
            send[:self.P] = op
        if run_side:
            stream.wait_stream(torch.cuda.current_stream(op.device))
            ctx = torch.cuda.stream(stream)
        else:
            ctx = _Null()
        with ctx:
            recv = torch.empty_like(send)
            all_to_all_rows(recv, send, group)
            if op.is_cuda:
                from ..ops.native import native

                tot = torch.empty((blk, 8), dtype=torch.int32, device=op.device)
                pref = torch.empty((size * blk, 7), dtype=torch.int32, device=op.device) if want_prefix else None
                native().sweep_block_reduce(recv, size, dtype == torch.bfloat16, tot, pref)
            else:
                tot, pref = block_reduce_rows(recv, size, dtype, want_prefix)
            total = torch.empty((size * blk, 8), dtype=torch.int32, device=op.device)
            all_gather_rows(total, tot, group)
            self._total = total[:self.P]
            if run_side:
                self._ev_total = torch.cuda.Event()
                self._ev_total.record(stream)
        self._pref = pref
        self._blk = blk
        self._group = group
        self._stream = stream if run_side else None

    def send_prefix(self, gate=None) -> None:
        """Enqueue the deferred all-to-all that returns every rank its prefix (on the
        collective stream, after ``gate(stream)`` -- the DP merge passes a wait on the next
        rating's tail, so the exchange does not compete with the rating's start)."""
        if self._pref is None or self._prefix is not None:
            return
        st = self._stream
        with (torch.cuda.stream(st) if st is not None else _Null()):
            if st is not None and gate is not None:
                gate(st)
            back = torch.empty((self.size * self._blk, 7), dtype=torch.int32, device=self._pref.device)
            all_to_all_rows(back, self._pref, self._group)
            self._prefix = back[:self.P]
            if st is not None:
                self._ev_prefix = torch.cuda.Event()
                self._ev_prefix.record(st)

    def total(self) -> torch.Tensor:
        """[P, 8] words of the summed operands; the current stream waits for them."""
        if self._ev_total is not None:
            cur = torch.cuda.current_stream(self._total.device)
            cur.wait_event(self._ev_total)
            self._total.record_stream(cur)
        return self._total

    def prefix(self) -> Optional[torch.Tensor]:
        """[P, 7] words of this rank's exclusive prefix; the current stream waits for it
        (``send_prefix`` first, or it is sent now, ungated)."""
        self.send_prefix()
        if self._prefix is not None and self._ev_prefix is not None:
            cur = torch.cuda.current_stream(self._prefix.device)
            cur.wait_event(self._ev_prefix)
            self._prefix.record_stream(cur)
        return self._prefix


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def all_reduce_sum(t: torch.Tensor, group=None, async_op: bool = False):
    """SUM all-reduce in place; gloo + device tensor goes through the host.
    Returns a work handle (``async_op``) or None."""
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def time_all_reduce(t: torch.Tensor, group=None, iters: int = 3) -> float:
    """Milliseconds per SUM all-reduce of ``t`` (one untimed warm-up, then the mean
    of ``iters``), the MAX over ranks -- so every rank takes the same decision from
    it.  A collective: every rank of the group must call it.  ``t`` is overwritten."""
    _, size = world(group)
    if size <= 1:
        return 0.0
    all_reduce_sum(t, group)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            all_reduce_sum(t, group)
        b.record()
        torch.cuda.synchronize(t.device)
        ms = a.elapsed_time(b) / iters
    else:
        import time

        t0 = time.perf_counter()
        for _ in range(iters):
            all_reduce_sum(t, group)
        ms = (time.perf_counter() - t0) * 1e3 / iters
    m = torch.tensor([ms], dtype=torch.float64, device=t.device if not _staged(t, group) else "cpu")
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return float(m.item())


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, torch.device]:
    """Initialise the default group from the torchrun environment (no-op for one
    process).  Returns (rank, world_size, device).  ``backend`` (default
    ``ANA_DIST_BACKEND``, else nccl = RCCL on a GPU): with ``gloo`` on a GPU box the ranks
    still rate on the device -- several may share one GPU (a rehearsal) -- and the
    collectives stage their tensors through the host (``_staged``)."""
    rank = int(os.environ.get("RANK", "0"))
    size = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or os.environ.get("ANA_DIST_BACKEND") or None
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        ngpu = torch.cuda.device_count()
        local = local % ngpu if backend == "gloo" and ngpu else local
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(local)
    if size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if use_gpu and backend in (None, "nccl"):
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend or "gloo")
    return rank, size, dev


def shard(n: int, rank: int, size: int) -> Tuple[int, int]:
    """[lo, hi) of rank's contiguous block of n items (sizes differ by <= 1)."""
    base, extra = divmod(int(n), int(size))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def broadcast_roster(roster, src: int = 0, group=None) -> None:
    """C3: make every rank's replica equal to ``src``'s (state + attributes)."""
    _, size = world()
    if size <= 1:
        return
    for t in (roster.state, roster.attrs):
        if _staged(t, group):
            h = t.cpu()
            dist.broadcast(h, src=src, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src, group=group)


def reduce_counts(counts: Dict[str, float], device, group=None, op: str = "sum") -> Dict[str, float]:
    """C4: reduce a dict of scalar metrics over ranks (same keys on every rank
    are not required: the key set is unioned first)."""
    _, size = world()
    if size <= 1:
        return dict(counts)
    keys = sorted(counts)
    gathered = [None] * size
    dist.all_gather_object(gathered, keys, group=group)
    keys = sorted(set(k for ks in gathered for k in ks))
    t = torch.tensor([float(counts.get(k, 0.0)) for k in keys], dtype=torch.float64, device=device)
    if _staged(t, group):
        t = t.cpu()
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=group)
    return {k: float(v) for k, v in zip(keys, t.cpu().tolist())}
