#!/usr/bin/python3
"""Drop-in ``worker`` entry point (/root/reference/worker.py).

Same environment variables and defaults as the reference (``RABBITMQ_URI``,
``DATABASE_URI``, ``BATCHSIZE``, ``CHUNKSIZE``, ``IDLE_TIMEOUT``, ``QUEUE``,
``DOCRUNCHMATCH``, ``CRUNCH_QUEUE``, ``DOTELESUCKMATCH``, ``TELESUCK_QUEUE``,
``DOSEWMATCH``, ``SEW_QUEUE``) plus ``ENGINE=python|native`` and
``QUARANTINE``; same module-level functions (``connect``, ``newjob``,
``try_process``, ``process``).  The work is done by
:class:`analyzer_amd.runtime.worker.Worker`.

    python3 worker.py                      # consume QUEUE until idle
    python3 worker.py --synthetic 1000     # config 1: populate + consume 1k 3v3 matches
    python3 worker.py --synthetic 100000 --replicas 8   # 8 worker processes on one queue

Without pika / a MySQL driver in this image, ``RABBITMQ_URI`` defaults to the
in-process broker (``memory://``) and ``DATABASE_URI`` to the in-process store;
``DATABASE_URI=sqlite:///path`` persists the reference's tables in SQLite.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from analyzer_amd.config import WorkerConfig
from analyzer_amd.runtime.worker import Worker
from analyzer_amd.utils.log import InfoFilter, get_logger  # noqa: F401  (public names)

_env = dict(os.environ)
_env.setdefault("RABBITMQ_URI", "memory://")
CONFIG = WorkerConfig.from_env(_env)

RABBITMQ_URI = CONFIG.rabbitmq_uri
DATABASE_URI = CONFIG.database_uri
BATCHSIZE = CONFIG.batchsize
CHUNKSIZE = CONFIG.chunksize
IDLE_TIMEOUT = CONFIG.idle_timeout
QUEUE = CONFIG.queue
DOCRUNCHMATCH = CONFIG.docrunchmatch
CRUNCH_QUEUE = CONFIG.crunch_queue
DOTELESUCKMATCH = CONFIG.dotelesuckmatch
TELESUCK_QUEUE = CONFIG.telesuck_queue
DOSEWMATCH = CONFIG.dosewmatch
SEW_QUEUE = CONFIG.sew_queue

logger = get_logger()
_worker = Worker(CONFIG)


def connect():
    """Open the store and the broker, declare queues, start consuming QUEUE."""
    return _worker.connect()


def newjob(ch, method, properties, body):
    return _worker.newjob(ch, method, properties, body)


def try_process():
    return _worker.try_process()


def process():
    return _worker.process()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--synthetic", type=int, default=0, help="populate and enqueue N synthetic matches")
    ap.add_argument("--players", type=int, default=0, help="synthetic roster size (default 2*N)")
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--replicas", type=int, default=0,
                    help="N >= 1: a shared broker (tcp://) and N worker processes on QUEUE, one per GPU, "
                         "over one store file (analyzer_amd/runtime/replicas.py); 0: this process alone")
    args = ap.parse_args(argv)
    if args.replicas >= 1:
        from analyzer_amd.runtime.replicas import run_replicas

        res = run_replicas(args.replicas, synthetic=args.synthetic, players=args.players,
                           team_size=args.team_size, seed=args.seed)
        print(json.dumps(res), flush=True)
        return 0 if res["ok"] else 1
    connect()
    if args.synthetic:
        from analyzer_amd.runtime.source import populate, publish

        matches = populate(_worker.store, args.synthetic, args.players or 2 * args.synthetic,
                           team_size=args.team_size, seed=args.seed)
        publish(_worker.channel, QUEUE, [m.api_id for m in matches])
    t0 = time.perf_counter()
    _worker.start_consuming()
    dt = time.perf_counter() - t0
    st = _worker.stats
    print(json.dumps({"matches": st.matches, "messages": st.messages, "batches": st.batches,
                      "failed_batches": st.failed_batches, "quarantined": st.quarantined,
                      "acked": st.acked, "nacked": st.nacked, "cas_retries": st.cas_retries, "seconds": dt,
                      "matches_per_s": st.matches / dt if dt > 0 else None,
                      "engine": CONFIG.engine}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
