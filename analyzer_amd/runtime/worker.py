"""The rating worker: ingest -> micro-batch -> rate -> commit -> ack -> fan-out
(/root/reference/worker.py).

Same observable protocol as the reference:

* ``connect()`` opens the store and the broker, declares ``QUEUE``,
  ``QUEUE_failed``, ``CRUNCH_QUEUE`` and ``TELESUCK_QUEUE`` (durable), sets
  ``prefetch_count=BATCHSIZE`` and consumes ``QUEUE`` (worker.py:85-92);
* ``newjob`` appends the delivery and arms ONE ``IDLE_TIMEOUT`` timer on the
  first message of a batch -- a max-latency bound, not reset by later
  messages -- and flushes at ``BATCHSIZE`` (worker.py:95-101);
* ``process`` dedups the bodies (match api ids), loads the matches ordered by
  ``created_at`` in chunks of ``CHUNKSIZE``, rates them in order and commits
  once (worker.py:169-199);
* ``try_process`` acks every delivery on success and fans out: ``notify``
  header -> ``"analyze_update"`` on ``amq.topic``; ``DOCRUNCHMATCH`` /
  ``DOSEWMATCH`` forward the body; ``DOTELESUCKMATCH`` publishes every asset
  url of the match with a ``match_api_id`` header (worker.py:103-166).  On
  failure every body goes to ``QUEUE_failed`` with its properties and is
  nacked without requeue (worker.py:108-120).

Deliberate, documented differences:

* ``ENGINE=native`` rates the whole batch with one launch of the batched
  engine instead of per-object Python: against a device-resident roster with
  one HIP-graph replay per batch (runtime/resident.py; ``RESIDENT=false``
  rebuilds the roster from the batch's objects instead, runtime/batch.py);
* ``QUARANTINE=true`` (default) isolates the matches the reference would raise
  on (tier None/30, sigma 0, empty roster, non-finite result): only their
  deliveries go to ``QUEUE_failed``; the rest of the batch commits.
  ``QUARANTINE=false`` restores the all-or-nothing batch of the reference;
* a delivery without headers is simply not notified (the reference raises
  AttributeError there and kills the consumer, worker.py:132);
* ``SEW_QUEUE`` is declared when ``DOSEWMATCH`` is on (the reference forwards to
  a queue it never declares, which a broker silently drops);
* ``DOTELEMETRY=true`` (with ``ENGINE=native``) aggregates per-event telemetry
  into ``participant_stats`` in the same launch as the rating (K8 fused mode,
  BASELINE config 4), on every store (on the reflected SQLAlchemy store through
  its columnar batch path).  The reference only forwards asset URLs
  (worker.py:148-161); here ``TELEMETRY_SOURCE`` names an ANATEL01 file of the
  downloaded events keyed by match api id (ops/telemetry.TelemetrySource,
  ``python -m analyzer_amd.ops.telemetry convert`` builds one from JSON lines).
  Without it the events are synthetic, and synthetic stats are never persisted
  into a real database: with a ``DATABASE_URI`` other than the in-process
  ``memory://`` / ``columnar://`` stores, ``connect`` refuses ``DOTELEMETRY``
  unless ``SYNTHETIC_TELEMETRY=true`` says the run is a benchmark.

Per-batch counters (matches rated/afk/invalid/unsupported/quarantined, timing)
are kept in ``stats`` and logged as one JSON line per batch (SURVEY §5 metrics).
"""
from __future__ import annotations

import json
import logging
import os
import random
import time
from operator import attrgetter

import numpy as np
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from ..config import RaterConfig, WorkerConfig
from ..models.match_rater import MatchRater
from ..utils.log import get_logger
from ..utils.trace import trace_range
from . import broker as B
from .store import open_store

logger = get_logger()


@dataclass
class WorkerStats:
    batches: int = 0
    failed_batches: int = 0
    messages: int = 0
    matches: int = 0
    quarantined: int = 0
    acked: int = 0
    nacked: int = 0
    published: Dict[str, int] = field(default_factory=dict)
    seconds: float = 0.0
    cas_retries: int = 0  # batches rated again after a versioned write conflict

    def bump(self, key: str, n: int = 1) -> None:
        self.published[key] = self.published.get(key, 0) + n


class MatchError(Exception):
    """A match the reference rater would raise on."""


class Worker:
    def __init__(self, cfg: Optional[WorkerConfig] = None, store=None, broker=None,
                 rater_cfg: Optional[RaterConfig] = None, clock: Optional[Callable[[], float]] = None,
                 object_rater=None):
        self.cfg = cfg or WorkerConfig.from_env()
        self.rater_cfg = rater_cfg or RaterConfig.from_env()
        self.store = store
        self.rabbit = broker
        self.clock = clock
        self.channel = None
        self.queue = Deliveries()
        self.timer = None
        self.stats = WorkerStats()
        self.failed_ids: List[str] = []
        self._python_rater = MatchRater(self.rater_cfg)
        self._object_rater = object_rater  # runtime.batch.ObjectBatchRater, built lazily
        self._tele_source = None
        self._pipe = False
        self._inflight: Optional[_InFlight] = None  # launched, not yet committed / acked
        self._flush = None                          # timer completing it when no batch follows

    # ------------------------------------------------------------ connect (W3/W4)
    def connect(self) -> "Worker":
        if self.cfg.dotelemetry and not self.cfg.synthetic_telemetry and not self.cfg.telemetry_source:
            uri = self.cfg.database_uri or ""
            if uri and not uri.startswith(("memory:", "columnar:")):  # in-process stores only
                raise ValueError("DOTELEMETRY without TELEMETRY_SOURCE aggregates SYNTHETIC telemetry: "
                                 "refusing to write it into %s; point TELEMETRY_SOURCE at an event "
                                 "file, or set SYNTHETIC_TELEMETRY=true for a benchmark run" % uri)
        if self.store is None:
            # no DATABASE_URI: an in-process store -- columnar for the native engine
            # (no per-object work at all), the object graph for the Python engine
            uri = self.cfg.database_uri or ("columnar://" if self.cfg.engine == "native" else None)
            self.store = open_store(uri)
        if (self.cfg.dotelemetry and type(self.store).__name__ == "SqlAlchemyStore"
                and not (self.cfg.engine == "native" and not self.cfg.skip_rated)):
            # the reflected store's participant_stats are written by the columnar batch
            # path (runtime/sqla.py load_batch / commit); its ORM relationships are read-only
            raise ValueError("DOTELEMETRY on a SQLAlchemy store needs the columnar path "
                             "(ENGINE=native, SKIP_RATED=false)")
        if self.rabbit is None:
            self.rabbit = B.connect(self.cfg.rabbitmq_uri, clock=self.clock)
        ch = self.rabbit.channel()
        for q in (self.cfg.queue, self.cfg.failed_queue, self.cfg.crunch_queue, self.cfg.telesuck_queue):
            ch.queue_declare(queue=q, durable=True)
        if self.cfg.dosewmatch:
            ch.queue_declare(queue=self.cfg.sew_queue, durable=True)
        self._pipe = self._pipelined()
        # pipelined: batch i+1 is delivered and launched before batch i is acked
        ch.basic_qos(prefetch_count=self.cfg.batchsize * (2 if self._pipe else 1))
        if hasattr(ch, "_deliver_bulk"):  # the in-process broker: whole prefetch windows per call
            ch.basic_consume(self.newjob, queue=self.cfg.queue, bulk_callback=self.newjobs)
        else:
            ch.basic_consume(self.newjob, queue=self.cfg.queue)
        self.channel = ch
        return self

    # ------------------------------------------------------------ batcher (W5)
    def newjob(self, _ch, method, properties, body) -> None:
        self.queue.append(method, properties, body)
        if self.timer is None:
            self.timer = self.rabbit.add_timeout(self.cfg.idle_timeout, self.try_process)
        if len(self.queue) == self.cfg.batchsize:
            self.try_process()

    def newjobs(self, _ch, tags, messages) -> None:
        """``newjob`` for a run of deliveries (the in-process broker's bulk path:
        a range of delivery tags and their messages): the same batches -- the
        timer armed by the first message of a batch, a flush at exactly
        BATCHSIZE -- without one Python call per message."""
        i, n, cap = 0, len(messages), self.cfg.batchsize
        while i < n:
            if self.timer is None:
                self.timer = self.rabbit.add_timeout(self.cfg.idle_timeout, self.try_process)
            take = min(n - i, cap - len(self.queue))
            self.queue.extend(tags[i:i + take], messages[i:i + take])
            i += take
            if len(self.queue) == cap:
                self.try_process()

    # ------------------------------------------------------------ ack / fan-out (W6)
    def try_process(self) -> None:
        if self.timer is not None:
            self.rabbit.remove_timeout(self.timer)
            self.timer = None
        batch, self.queue = self.queue, Deliveries()
        if batch and self.cfg.fault_exit_after and self.stats.batches >= self.cfg.fault_exit_after:
            logger.error("injected fault (FAULT_EXIT_AFTER=%d): exiting with %d deliveries unacked",
                         self.cfg.fault_exit_after, len(batch))
            os._exit(17)
        if self._pipe:
            self._pipeline_step(batch)
            return
        if not batch:
            return
        t0 = time.perf_counter()
        try:
            failed = set(self.process(batch))
        except Exception as e:  # the whole batch goes to the failed queue (worker.py:110-120)
            self._fail_batch(batch, e, t0)
            return
        self._settle(batch, failed, t0)

    def _fail_batch(self, batch, e: Exception, t0: float) -> None:
        logger.error(e)
        for meth, prop, body in batch:
            self._publish("", self.cfg.failed_queue, body, prop)
            self.channel.basic_nack(meth.delivery_tag, requeue=False)
            self.stats.nacked += 1
        self.stats.failed_batches += 1
        self.stats.seconds += time.perf_counter() - t0

    def _settle(self, batch, failed, t0: float) -> None:
        """Ack a processed batch and fan out (worker.py:122-166)."""
        logger.info("acking batch")
        session = self.store.session() if self.cfg.dotelesuckmatch else None
        try:
            with trace_range("ack"):
                # every delivery of the batch is settled: the quarantined ones are
                # nacked, then ONE basic_ack(multiple=True) of the highest good tag
                # settles the rest -- what the reference's per-message acks do, in one
                # frame (a later batch in flight holds only higher tags)
                if failed:
                    ok_tags = []
                    for meth, prop, body in batch:
                        if _decode(body) in failed:  # quarantined match
                            self._publish("", self.cfg.failed_queue, body, prop)
                            self.channel.basic_nack(meth.delivery_tag, requeue=False)
                            self.stats.nacked += 1
                        else:
                            ok_tags.append(meth.delivery_tag)
                else:
                    ok_tags = batch.tags
                if ok_tags:
                    self.channel.basic_ack(max(ok_tags), multiple=True)
                    self.stats.acked += len(ok_tags)
                fanout = self.cfg.docrunchmatch or self.cfg.dosewmatch or self.cfg.dotelesuckmatch
                for meth, prop, body in (batch if fanout or batch.any_headers() else ()):
                    headers = (prop.headers if prop is not None else None) or {}
                    if not fanout and not headers:
                        continue
                    mid = _decode(body)
                    if mid in failed:
                        continue
                    if headers.get("notify"):
                        self._publish("amq.topic", headers.get("notify"), b"analyze_update", None)
                    if self.cfg.docrunchmatch:
                        self._publish("", self.cfg.crunch_queue, body, prop)
                    if self.cfg.dosewmatch:
                        self._publish("", self.cfg.sew_queue, body, prop)
                    if self.cfg.dotelesuckmatch:
                        for asset in session.assets(mid):
                            self._publish("", self.cfg.telesuck_queue, asset.url,
                                          B.BasicProperties(headers={"match_api_id": asset.match_api_id}))
        finally:
            if session is not None:
                session.close()
        self.stats.batches += 1
        self.stats.seconds += time.perf_counter() - t0

    # ------------------------------------------------------------ pipelined batches
    # ENGINE=native on an in-process columnar store keeps TWO batches in flight:
    # batch i+1 is loaded, encoded and launched (runtime/resident.launch_batch)
    # before batch i is finished, committed and acked, so the device work and the
    # copies back of one batch overlap the host stages of the other.  Launches are
    # stream-ordered, so batch i+1 rates from batch i's results exactly as the
    # serial worker would; commits and acks stay in batch order.  When batch i
    # fails as a whole (QUARANTINE=false error, failed commit), batch i+1 is
    # rolled back on the device first, then batch i, and batch i+1 is launched
    # again from the restored state -- the serial path's outcome (test:
    # tests/test_worker.py::test_pipelined_worker_is_the_serial_worker).  A batch
    # in flight with no successor is completed by a 1-ms timer.
    def _pipelined(self) -> bool:
        return bool(self.cfg.pipeline and self.cfg.engine == "native" and self.cfg.resident
                    and not self.cfg.skip_rated and getattr(self.store, "concurrent_sessions", False))

    def _pipeline_step(self, batch) -> None:
        if self._flush is not None:
            self.rabbit.remove_timeout(self._flush)
            self._flush = None
        nxt = self._launch(batch) if batch else None
        prev, self._inflight = self._inflight, None
        if prev is not None:
            self._complete(prev, later=nxt)
        if nxt is None:
            return
        if nxt.error is not None:  # load / launch failed: the whole batch fails
            self._fail_batch(nxt.batch, nxt.error, nxt.t0)
            return
        self._inflight = nxt
        self._flush = self.rabbit.add_timeout(min(self.cfg.idle_timeout, 0.001), self._flush_inflight)

    def _flush_inflight(self) -> None:
        self._flush = None
        prev, self._inflight = self._inflight, None
        if prev is not None:
            self._complete(prev)

    def _launch(self, batch, fl: Optional["_InFlight"] = None) -> "_InFlight":
        t0 = time.perf_counter()
        if fl is None:
            fl = _InFlight(batch, t0)
            fl.ids = batch.match_ids()
            self.stats.messages += len(batch)
        undo_before = None
        try:
            if fl.session is None:
                fl.session = self.store.session()
                with trace_range("load", ids=len(fl.ids)):
                    fl.mb = fl.session.load_batch(fl.ids, self.cfg.chunksize)
            # the telemetry seed of the serial worker: batches committed before this one
            seed_batches = self.stats.batches + (1 if self._inflight is not None else 0)
            self._inject_faults(fl.mb)
            undo_before = getattr(self._batched(), "_undo", None)
            with trace_range("rate", matches=len(fl.mb), engine="native"):
                fl.pending = self._batched().launch_batch(fl.mb, fl.session.fetch_players,
                                                          telemetry=self._telemetry_spec(seed_batches),
                                                          stage=getattr(fl.session, "stage_players", None))
        except Exception as e:
            if fl.session is not None:
                fl.session.rollback()
                fl.session.close()
            # a launch that failed after its undo snapshot (e.g. in the copies back)
            # must not leave its updates in the device roster: the serial path's
            # process() rolls them back the same way
            rater = self._object_rater
            undo = getattr(rater, "_undo", None)
            if undo is not None and undo is not undo_before and hasattr(rater, "rollback"):
                rater.rollback()  # this batch's snapshot, never the batch still in flight
            fl.error, fl.pending = e, None
        fl.seconds += time.perf_counter() - t0
        return fl

    def _complete(self, fl: "_InFlight", later: Optional["_InFlight"] = None) -> None:
        t0 = time.perf_counter()
        rater, counts = self._batched(), {}
        try:
            status = rater.finish_batch(fl.pending)
            quarantined = self._statuses(fl.mb, status, counts)
            with trace_range("commit"):
                fl.session.commit()
        except Exception as e:
            if later is not None and later.pending is not None:
                rater.rollback(later.pending)  # the later batch first: it rated on top of this one
            fl.session.rollback()
            rater.rollback(fl.pending)
            fl.session.close()
            self._fail_batch(fl.batch, e, t0 - fl.seconds)
            if later is not None and later.pending is not None:
                self._launch(later.batch, later)  # again, from the restored state
            return
        fl.session.close()
        fl.pending.undo = None
        self.stats.matches += len(fl.mb)
        self.stats.quarantined += len(quarantined)
        self.failed_ids += quarantined
        if logger.isEnabledFor(logging.INFO):
            logger.info(json.dumps({"batch": self.stats.batches, "messages": len(fl.batch),
                                    "matches": len(fl.mb), "engine": self.cfg.engine,
                                    "quarantined": len(quarantined), **counts}))
        self._settle(fl.batch, set(quarantined), t0 - fl.seconds)

    def _publish(self, exchange: str, key: str, body, props) -> None:
        self.channel.basic_publish(exchange=exchange, routing_key=key, body=body, properties=props)
        self.stats.bump(key if exchange == "" else exchange)

    # ------------------------------------------------------------ process (W7)
    def process(self, batch=None) -> List[str]:
        """Rate one batch; returns the api ids of quarantined matches.  Raises
        (after rolling back) when the batch must fail as a whole."""
        batch = self.queue if batch is None else batch
        logger.info("analyzing batch %s", str(len(batch)))
        ids = batch.match_ids() if isinstance(batch, Deliveries) else list(set(_decode(b) for _, _, b in batch))
        self.stats.messages += len(batch)
        from .store import WriteConflict

        attempt = 0
        lock_first = os.environ.get("CAS_LOCK") == "always"
        while True:
            try:
                # a retried batch takes the store's write lock before it reads its players
                # (SqliteSession.lock): it cannot lose the race twice
                matches, quarantined, counts = self._process_once(ids, locked=attempt > 0 or lock_first)
                break
            except WriteConflict as e:
                # another replica committed some of this batch's players since they were
                # read: everything was rolled back -- rate the batch again from fresh rows
                attempt += 1
                self.stats.cas_retries += 1
                if attempt > self.cfg.cas_retries:
                    raise
                logger.info("batch write conflict (%s): retry %d", e, attempt)
                time.sleep(random.uniform(0.0, 0.002 * min(attempt, 10)))
        self.stats.matches += len(matches)
        self.stats.quarantined += len(quarantined)
        self.failed_ids += quarantined
        if logger.isEnabledFor(logging.INFO):
            logger.info(json.dumps({"batch": self.stats.batches, "messages": len(batch),
                                    "matches": len(matches), "engine": self.cfg.engine,
                                    "quarantined": len(quarantined), **counts}))
        return quarantined

    def _process_once(self, ids, locked: bool = False):
        """One attempt at a batch: load, rate, commit (all rolled back on an exception);
        ``locked``: under the store's write lock from the start (stores that have one)."""
        session = self.store.session()
        if locked and hasattr(session, "lock"):
            session.lock()
        quarantined: List[str] = []
        counts: Dict[str, int] = {}
        try:
            if self.cfg.engine == "native" and not self.cfg.skip_rated and hasattr(session, "load_batch"):
                # columnar path: no per-object work (runtime/columnar.py); without
                # RESIDENT the batch's players are all re-read from the store
                if not self.cfg.resident or getattr(self.store, "versioned", False):
                    # (versioned writes need the version of every player row read)
                    self._batched().resident.reset()
                with trace_range("load", ids=len(ids)):
                    mb = session.load_batch(ids, self.cfg.chunksize)
                with trace_range("rate", matches=len(mb), engine="native"):
                    quarantined = self._rate_batch(mb, session, counts)
                matches = mb.ids
            else:
                with trace_range("load", ids=len(ids)):
                    matches = list(session.load_matches(ids, self.cfg.chunksize))
                if self.cfg.skip_rated:
                    fresh = [m for m in matches if m.trueskill_quality is None]
                    if len(fresh) != len(matches):
                        counts["skipped_rated"] = len(matches) - len(fresh)
                    matches = fresh
                with trace_range("rate", matches=len(matches), engine=self.cfg.engine):
                    if self.cfg.engine == "native" and self._batched().supports(matches):
                        quarantined = self._rate_native(session, matches, counts)
                    else:
                        quarantined = self._rate_python(session, matches, counts)
                        self._forget_resident(matches)
            with trace_range("commit"):
                session.commit()
            if self._object_rater is not None and hasattr(self._object_rater, "commit"):
                self._object_rater.commit()
        except Exception:
            session.rollback()
            if self._object_rater is not None and hasattr(self._object_rater, "rollback"):
                self._object_rater.rollback()  # the device roster too
            raise
        finally:
            session.close()
        return matches, quarantined, counts

    def _rate_python(self, session, matches, counts) -> List[str]:
        bad = []
        for match in matches:
            sp = session.savepoint(match) if self.cfg.quarantine else None
            try:
                if match.api_id in self.cfg.fault_poison:
                    raise FloatingPointError("injected fault (FAULT_POISON)")
                self._python_rater.rate_match(match)
                counts["rated"] = counts.get("rated", 0) + 1
            except (KeyError, ValueError, FloatingPointError, ZeroDivisionError, IndexError,
                    TypeError) as e:
                if not self.cfg.quarantine:
                    raise
                session.restore(match, sp)
                logger.error("quarantined match %s: %r", match.api_id, e)
                bad.append(match.api_id)
        return bad

    def _forget_resident(self, matches) -> None:
        """Players the Python engine just rated: the device-resident copies are
        stale, so their next native batch re-reads them from the store."""
        res = getattr(self._object_rater, "resident", None)
        if res is None or not hasattr(res, "forget"):
            return
        res.forget({p.player[0].api_id for m in matches for r in m.rosters for p in r.participants
                    if p.player})

    def _batched(self):
        if self._object_rater is None:
            from ..ops.rate import BatchRater

            if self.cfg.resident or getattr(self.store, "columnar_batches", False):
                from .resident import ResidentBatchRater
                self._object_rater = ResidentBatchRater(BatchRater(self.rater_cfg),
                                                        capacity=self.cfg.batchsize)
            else:
                from .batch import ObjectBatchRater
                self._object_rater = ObjectBatchRater(BatchRater(self.rater_cfg))
        return self._object_rater

    def _telemetry_spec(self, batches_before: Optional[int] = None):
        if not self.cfg.dotelemetry:
            return None
        if self.cfg.telemetry_source:  # real events, opened once
            if self._tele_source is None:
                from ..ops.telemetry import TelemetrySource
                self._tele_source = TelemetrySource(self.cfg.telemetry_source)
            return self._tele_source
        from ..ops.telemetry import TelemetrySpec
        lo, hi = (int(x) for x in self.cfg.telemetry_events.split(","))
        before = self.stats.batches if batches_before is None else batches_before
        return TelemetrySpec(seed=before + 1, min_events=lo, max_events=hi)

    def _rate_batch(self, batch, session, counts) -> List[str]:
        from ..ops import rate as R

        if len(batch) == 0:
            return []
        self._inject_faults(batch)
        status = self._batched().rate_batch(batch, session.fetch_players, telemetry=self._telemetry_spec(),
                                            stage=getattr(session, "stage_players", None))
        return self._statuses(batch, status, counts)

    def _inject_faults(self, batch) -> None:
        """FAULT_POISON on a columnar batch: the poisoned matches lose their
        participants, so the kernels report an empty roster -- a failed match that
        leaves the state untouched, quarantined like any other."""
        if self.cfg.fault_poison:
            for i, mid in enumerate(batch.ids):
                if mid in self.cfg.fault_poison:
                    batch.n[i] = 0

    def _statuses(self, batch, status, counts) -> List[str]:
        """Count a rated batch's statuses; its quarantined match ids (raises with
        QUARANTINE=false)."""
        from ..ops import rate as R

        num = np.bincount(status, minlength=256)
        for v in np.flatnonzero(num).tolist():
            name = R.STATUS_NAMES.get(v, str(v))
            counts[name] = counts.get(name, 0) + int(num[v])
        bad = ([batch.ids[i] for i in np.flatnonzero(_BAD_STATUS[status]).tolist()]
               if num[_BAD_STATUS].any() else [])
        if bad and not self.cfg.quarantine:
            raise MatchError("%d match(es) failed to rate (first: %s)" % (len(bad), bad[0]))
        return bad

    def _rate_native(self, session, matches, counts) -> List[str]:
        from ..ops import rate as R

        bad = []
        if self.cfg.fault_poison:  # injected faults: never rated, like a failed match
            bad = [m.api_id for m in matches if m.api_id in self.cfg.fault_poison]
            if bad:
                counts["fault_injected"] = len(bad)
                matches = [m for m in matches if m.api_id not in self.cfg.fault_poison]
        rater = self._batched()
        res = getattr(rater, "resident", None)
        if res is not None and (not self.cfg.resident or getattr(self.store, "versioned", False)):
            # a ResidentBatchRater on a columnar-capable store without RESIDENT (the
            # object path: SKIP_RATED, or a store without load_batch): the device rows
            # cached by api id would go stale against other replicas' commits, so the
            # batch's players are re-read from its objects, as ObjectBatchRater does
            res.reset()
        status = rater.rate(matches, telemetry=self._telemetry_spec()) if matches else []
        for m, s in zip(matches, status):
            name = R.STATUS_NAMES.get(s, str(s))
            counts[name] = counts.get(name, 0) + 1
            if s in R.ERROR_STATUSES or s == R.NOT_PROCESSED:
                bad.append(m.api_id)
        if bad and not self.cfg.quarantine:
            raise MatchError("%d match(es) failed to rate (first: %s)" % (len(bad), bad[0]))
        return bad

    # ------------------------------------------------------------ entry point (W9)
    def start_consuming(self, until: Optional[Callable[[], bool]] = None) -> None:
        self.rabbit.run(until=until)

    def run(self) -> None:
        self.connect()
        self.start_consuming()


class Deliveries:
    """A batch of deliveries as parallel lists (tags, properties, bodies);
    iterating yields the ``(method, properties, body)`` triples of the per-message
    callback, built only on the paths that need them (failures, fan-out)."""

    __slots__ = ("tags", "props", "bodies")

    def __init__(self):
        self.tags: List[int] = []
        self.props: List[Optional[B.BasicProperties]] = []
        self.bodies: List[bytes] = []

    def append(self, method, props, body) -> None:
        self.tags.append(method.delivery_tag)
        self.props.append(props)
        self.bodies.append(body)

    def extend(self, tags, messages) -> None:
        self.tags.extend(tags)
        self.props.extend([m.properties for m in messages])
        self.bodies.extend([m.body for m in messages])

    def __len__(self) -> int:
        return len(self.tags)

    def __iter__(self):
        for t, p, b in zip(self.tags, self.props, self.bodies):
            yield B.Method(t, ""), p, b

    def any_headers(self) -> bool:
        try:
            return any(map(_headers, self.props))
        except AttributeError:  # deliveries without properties
            return any(p is not None and p.headers for p in self.props)

    def match_ids(self) -> List[str]:
        """The deduplicated match api ids (bodies)."""
        try:
            return list(set(map(bytes.decode, self.bodies)))
        except TypeError:  # str / bytearray bodies
            return list(set(map(_decode, self.bodies)))


def _bad_status_table() -> np.ndarray:
    from ..ops import rate as R

    t = np.zeros(256, dtype=bool)
    t[list(R.ERROR_STATUSES) + [R.NOT_PROCESSED]] = True
    return t


_BAD_STATUS = _bad_status_table()


class _InFlight:
    """A pipelined batch between launch and ack."""

    def __init__(self, batch, t0: float):
        self.batch, self.t0 = batch, t0
        self.ids: List[str] = []
        self.session = self.mb = self.pending = self.error = None
        self.seconds = 0.0


_headers = attrgetter("headers")


def _decode(body) -> str:
    return str(body, "utf-8") if isinstance(body, (bytes, bytearray)) else str(body)
