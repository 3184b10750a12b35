"""Horizontal scale-out of the streaming worker: N worker processes on one queue
(SURVEY P1 "replica scale-out"; /root/reference/worker.py:91).

The reference scales by starting more ``worker.py`` processes against one RabbitMQ
queue (prefetch ``BATCHSIZE`` each) and one MySQL database.  ``run_replicas`` does
the same on one node: a ``BrokerServer`` (runtime/broker_net.py, ``tcp://``) stands
in for RabbitMQ, the store is a shared file (``DATABASE_URI=sqlite:///path`` or any
SQLAlchemy URL), and each replica is a child ``worker.py`` process pinned to one GPU
(``HIP_VISIBLE_DEVICES``; on the host mirror they share the CPU).  With a real
RabbitMQ, start the replicas the same way with ``RABBITMQ_URI=amqp://...``.

Delivery semantics are the reference's: each message is delivered to one replica at a
time and redelivered if that replica dies before acking it (at-least-once).  Player rows
are NOT raced on: the reference's replicas read, rate and write back with no locking,
so two replicas rating matches that share a player overwrite each other's update
(worker.py:174-194).  Here the store's player rows carry a version (runtime/store.py):
every write is a compare-and-set on the version the batch read, and a batch that loses
the race is rolled back and rated again from the fresh rows (runtime/worker.py
``process``; counted as ``cas_retries``) -- no update is lost, and the committed
batches are equivalent to rating them one after another in commit order
(tests/test_replicas.py replays the commit log).  ``racy=True`` (PLAYER_CAS=0) restores
the reference's behaviour for comparison.
The launcher prints one JSON line: per-replica and total matches, acks and rate, and
the broker's final counts.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional


def _visible_devices(env: Dict[str, str], n: int) -> List[str]:
    """The HIP_VISIBLE_DEVICES values the children may use: the entries of the
    parent's own HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES, which HIP also reads)
    when it runs under one (e.g. '4,5'), else 0..n-1 -- replica r gets entry r mod n,
    never a raw index outside the parent's set.  ROCR_VISIBLE_DEVICES is inherited by
    the children and HIP indexes within it, so there 0..n-1 is already right."""
    for key in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(key)
        if v:
            ids = [x.strip() for x in v.split(",") if x.strip()]
            if ids:
                return ids[:n] if n > 0 else ids
    return [str(i) for i in range(n)]


def _gpus() -> int:
    """Devices visible to the children (counting does not initialise the GPU here)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover - torch always present in this image
        return 0


def run_replicas(n: int, synthetic: int = 0, players: int = 0, team_size: int = 3, seed: int = 1,
                 database_uri: Optional[str] = None, queue: Optional[str] = None,
                 env: Optional[Dict[str, str]] = None, timeout: float = 600.0,
                 worker_py: Optional[str] = None,
                 replica_env: Optional[Dict[int, Dict[str, str]]] = None,
                 first_alone_until_acked: int = 0, racy: bool = False) -> Dict[str, object]:
    """Start a broker and ``n`` worker replicas, optionally populating and enqueueing
    ``synthetic`` matches first; wait until every replica drained the queue and exited.
    ``replica_env``: extra environment per replica index (fault injection in tests);
    ``first_alone_until_acked``: start replica 0 alone and the others once the broker
    counted that many acks (a deterministic first consumer for tests)."""
    from ..config import WorkerConfig
    from .broker_net import BrokerServer
    from .source import populate
    from .store import open_store

    base = dict(os.environ if env is None else env)
    queue = queue or WorkerConfig.from_env(base).queue
    tmpdir = None
    if not database_uri:
        database_uri = base.get("DATABASE_URI") or ""
    if not database_uri or database_uri.startswith(("memory:", "columnar:")) or database_uri == "sqlite://":
        # replicas need one store they all see: a SQLite file
        tmpdir = tempfile.mkdtemp(prefix="ana_replicas_")
        database_uri = "sqlite:///" + os.path.join(tmpdir, "store.db")
    server = BrokerServer().start()
    ids: List[str] = []
    if synthetic:
        store = open_store(database_uri)
        matches = populate(store, synthetic, players or 2 * synthetic, team_size=team_size, seed=seed)
        ids = [m.api_id for m in matches]
        del store
        server.publish(queue, [i.encode() for i in ids])
    worker_py = worker_py or os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "worker.py")
    gpus = _gpus()
    procs = []
    t0 = time.perf_counter()
    for r in range(n):
        e = dict(base)
        e.update(RABBITMQ_URI=server.uri, DATABASE_URI=database_uri, QUEUE=queue, REPLICA=str(r))
        if racy:
            e["PLAYER_CAS"] = "0"
        e.update((replica_env or {}).get(r, {}))
        if gpus > 0:  # one replica per GPU (round-robin when there are more replicas)
            ids = _visible_devices(base, gpus)
            e["HIP_VISIBLE_DEVICES"] = ids[r % len(ids)]
        # output to files: a replica blocked on a full pipe would hold its deliveries
        fo, fe = tempfile.TemporaryFile("w+"), tempfile.TemporaryFile("w+")
        procs.append((subprocess.Popen([sys.executable, worker_py], env=e, stdout=fo, stderr=fe), fo, fe))
        if r == 0 and first_alone_until_acked:
            wait_until = time.monotonic() + timeout / 2
            while (server.stats()["acked"] < first_alone_until_acked and procs[0][0].poll() is None
                   and time.monotonic() < wait_until):
                time.sleep(0.05)
    results, codes = [], []
    deadline = time.monotonic() + timeout
    for p, fo, fe in procs:
        try:
            p.wait(timeout=max(1.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        codes.append(p.returncode)
        fo.seek(0)
        fe.seek(0)
        out, err = fo.read(), fe.read()
        fo.close()
        fe.close()
        line = [ln for ln in out.splitlines() if ln.startswith("{")]
        results.append(json.loads(line[-1]) if line else {"error": err[-2000:]})
    dt = time.perf_counter() - t0
    stats = server.stats()
    # messages neither acked nor dead-lettered when the last replica left (ready, or
    # held by a replica that exited without settling them): lost work -- the launcher
    # reports it and worker.py --replicas exits non-zero
    unsettled = server.in_flight(queue)
    server.close()
    total = sum(int(r.get("matches", 0)) for r in results)
    return {"replicas": n, "gpus": gpus, "matches": total, "enqueued": len(ids),
            "acked": sum(int(r.get("acked", 0)) for r in results),
            "nacked": sum(int(r.get("nacked", 0)) for r in results),
            "cas_retries": sum(int(r.get("cas_retries", 0) or 0) for r in results),
            "seconds": dt, "matches_per_s": total / dt if dt > 0 else None,
            "per_replica": [{"matches": r.get("matches"), "acked": r.get("acked"),
                             "matches_per_s": r.get("matches_per_s"), "error": r.get("error")} for r in results],
            "exit_codes": codes, "broker": stats, "unsettled": unsettled,
            "ok": unsettled == 0 and all(c == 0 for c in codes), "database_uri": database_uri}
