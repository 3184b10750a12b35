"""Process-group plumbing and small collectives.

One process per GPU, ``torch.distributed`` with backend ``nccl`` (RCCL on ROCm,
over xGMI) for device tensors and ``gloo`` for the CPU tests.  The reference has
no collectives at all: its replicas share state through MySQL rows and
messages through RabbitMQ (/root/reference/worker.py:44-46,85-92).

* ``init_from_env``  -- RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (torchrun).
* ``broadcast_roster`` (C3) -- the initial replicated roster from one rank.
* ``reduce_counts`` (C4) -- status counters and timings summed / maxed over ranks.
* ``shard`` -- contiguous block partition of a range (time-axis sharding, P1/P4).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, torch.device]:
    """Initialise the default group from the torchrun environment (no-op for one
    process).  Returns (rank, world_size, device)."""
    rank = int(os.environ.get("RANK", "0"))
    size = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(local)
    if size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if use_gpu:
            dist.init_process_group(backend or "nccl", device_id=dev)
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
    dist.broadcast(roster.state, src=src, group=group)
    dist.broadcast(roster.attrs, src=src, group=group)


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
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=group)
    return {k: float(v) for k, v in zip(keys, t.cpu().tolist())}
