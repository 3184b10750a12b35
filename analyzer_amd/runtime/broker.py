"""In-process message broker with the AMQP 0-9-1 semantics the worker relies on
(SURVEY W4-W6, L1').

The reference talks to RabbitMQ through ``pika.BlockingConnection``
(/root/reference/worker.py:85-92) and uses exactly this surface:

* ``queue_declare(queue, durable=True)``, ``basic_qos(prefetch_count=N)``,
  ``basic_consume(callback, queue=Q)`` and ``start_consuming()`` (a blocking,
  single-threaded delivery loop that also fires timers);
* ``add_timeout(seconds, callback)`` / ``remove_timeout(handle)`` on the
  connection (the batcher's max-latency flush, worker.py:98-99,105-107);
* ``basic_ack(tag)``, ``basic_nack(tag, requeue=False)`` and
  ``basic_publish(exchange, routing_key, body, properties)`` on the default
  exchange (queue name = routing key) and on ``amq.topic``.

``MemoryBroker`` implements that surface with the broker-side behaviour that
matters for correctness tests: at most ``prefetch_count`` unacknowledged
deliveries per consumer, redelivery of unacknowledged messages when a channel
closes (consumer death -> at-least-once), ``redelivered`` flags, messages to an
undeclared queue on the default exchange are dropped (AMQP routes them
nowhere -- the reference never declares ``SEW_QUEUE``, worker.py:87-90), and
topic-exchange bindings with ``*`` / ``#`` patterns.  Time comes from an
injectable clock so batching tests are deterministic.

``connect(uri)`` returns a MemoryBroker for ``memory://`` URIs and, for
``amqp://`` ones, a ``PikaBroker``: the same surface over a real
``pika.BlockingConnection`` (pika 0.10, the reference's pin, or 1.x).  This
image has no pika, so the adapter is tested against a fake pika
module of both API generations (tests/test_worker.py); against a live
RabbitMQ its parity is unpinned.
"""
from __future__ import annotations

import heapq
import itertools
import re
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, NamedTuple, Optional, Tuple


@dataclass
class BasicProperties:
    """``pika.BasicProperties`` subset: headers plus the delivery mode."""

    headers: Optional[Dict[str, object]] = None
    delivery_mode: Optional[int] = None
    content_type: Optional[str] = None


class Method(NamedTuple):
    """``pika.spec.Basic.Deliver`` subset (a named tuple: one is built per
    delivery, and a tuple costs a fraction of a class instance)."""

    delivery_tag: int
    routing_key: str
    exchange: str = ""
    redelivered: bool = False
    consumer_tag: str = ""


@dataclass
class Message:
    body: bytes
    properties: BasicProperties
    routing_key: str
    exchange: str = ""
    redelivered: bool = False
    queue: str = ""  # the queue holding it (set when routed)


class ManualClock:
    """Deterministic clock for tests: time only moves when ``advance`` is called."""

    def __init__(self, t0: float = 0.0):
        self.t = float(t0)

    def __call__(self) -> float:
        return self.t

    def advance(self, dt: float) -> None:
        self.t += float(dt)


def _topic_regex(pattern: str) -> "re.Pattern[str]":
    """AMQP topic pattern -> regex (``*`` = one word, ``#`` = zero or more words)."""
    words = []
    for w in pattern.split("."):
        words.append("#" if w == "#" else ("[^.]+" if w == "*" else re.escape(w)))
    rx = r"\.".join(words)
    rx = rx.replace(r"\.#", r"(?:\.[^.]+)*").replace(r"#\.", r"(?:[^.]+\.)*").replace("#", ".*")
    return re.compile("^" + rx + "$")


@dataclass
class _Queue:
    name: str
    durable: bool
    ready: Deque[Message] = field(default_factory=deque)


class Channel:
    """One consumer channel (the worker opens exactly one)."""

    def __init__(self, broker: "MemoryBroker", number: int):
        self.broker = broker
        self.number = number
        self.prefetch_count = 0  # 0 = unlimited (AMQP default)
        self.consumers: List[Tuple[str, Callable]] = []
        self.bulk: Dict[int, Callable] = {}  # consumer index -> bulk callback (in-process extension)
        self.unacked: Dict[int, Message] = {}  # delivery tag -> message (msg.queue: its queue)
        self._tags = itertools.count(1)
        self.is_open = True
        self.acked = 0
        self.nacked = 0

    # -------------------------------------------------------------- declare/qos
    def queue_declare(self, queue: str, durable: bool = False, **_) -> None:
        self.broker.declare(queue, durable)

    def queue_bind(self, queue: str, exchange: str, routing_key: str) -> None:
        self.broker.bind(queue, exchange, routing_key)

    def basic_qos(self, prefetch_count: int = 0, **_) -> None:
        self.prefetch_count = int(prefetch_count)

    def basic_consume(self, *args, **kwargs) -> str:
        """Both the pika 0.10 form ``basic_consume(callback, queue=Q)`` used by the
        reference (worker.py:92) and the 1.x form ``basic_consume(queue, callback)``."""
        queue = kwargs.get("queue")
        callback = kwargs.get("on_message_callback") or kwargs.get("consumer_callback")
        for a in args:
            if callable(a):
                callback = a
            elif isinstance(a, str) and queue is None:
                queue = a
        if queue is None or callback is None:
            raise TypeError("basic_consume needs a queue and a callback")
        if queue not in self.broker.queues:
            raise KeyError("NOT_FOUND - no queue '%s'" % queue)
        tag = "ctag%d.%d" % (self.number, len(self.consumers) + 1)
        if kwargs.get("bulk_callback") is not None:
            # in-process extension: deliver every deliverable message of the queue (up to
            # the prefetch window) in ONE call of bulk_callback(channel, tags, messages)
            # (a range of delivery tags, the Message objects) -- the same deliveries,
            # tags and order as one call per message, without the per-message Python
            # dispatch and Method objects
            self.bulk[len(self.consumers)] = kwargs["bulk_callback"]
        self.consumers.append((queue, callback))
        return tag

    # ------------------------------------------------------------- publish/ack
    def basic_publish(self, exchange: str = "", routing_key: str = "", body=b"",
                      properties: Optional[BasicProperties] = None, **_) -> None:
        if isinstance(body, str):
            body = body.encode("utf-8")
        self.broker.publish(exchange, routing_key, bytes(body), properties or BasicProperties())

    def basic_ack(self, delivery_tag: int = 0, multiple: bool = False) -> None:
        tags = self._settle(delivery_tag, multiple)
        if multiple and len(tags) == len(self.unacked):
            self.unacked.clear()
        else:
            for tag in tags:
                self.unacked.pop(tag)
        self.acked += len(tags)

    def basic_nack(self, delivery_tag: int = 0, multiple: bool = False, requeue: bool = True) -> None:
        for tag in self._settle(delivery_tag, multiple):
            msg = self.unacked.pop(tag)
            self.nacked += 1
            if requeue:
                msg.redelivered = True
                self.broker.queues[msg.queue].ready.appendleft(msg)
            else:
                self.broker.dead_lettered.append(msg)

    def basic_reject(self, delivery_tag: int, requeue: bool = True) -> None:
        self.basic_nack(delivery_tag, requeue=requeue)

    def _settle(self, delivery_tag: int, multiple: bool) -> List[int]:
        if multiple:
            if self.unacked and (delivery_tag == 0 or delivery_tag >= next(reversed(self.unacked))):
                return list(self.unacked)  # everything outstanding (tags are issued in order)
            # unacked is in delivery (= tag) order: the settled tags are a prefix
            tags = list(itertools.takewhile(lambda t: t <= delivery_tag, self.unacked))
        else:
            if delivery_tag not in self.unacked:
                raise KeyError("PRECONDITION_FAILED - unknown delivery tag %d" % delivery_tag)
            tags = [delivery_tag]
        return sorted(tags)

    # ---------------------------------------------------------------- delivery
    def _deliver_one(self) -> bool:
        if not self.is_open:
            return False
        if self.prefetch_count and len(self.unacked) >= self.prefetch_count:
            return False
        for qname, cb in self.consumers:
            q = self.broker.queues[qname]
            if q.ready:
                msg = q.ready.popleft()
                tag = next(self._tags)
                self.unacked[tag] = msg
                method = Method(tag, msg.routing_key, msg.exchange, msg.redelivered)
                cb(self, method, msg.properties, msg.body)
                return True
        return False

    def _deliver_bulk(self) -> int:
        """Deliveries to a bulk consumer (see basic_consume); 0 if none is ready."""
        if not self.is_open or not self.bulk:
            return 0
        room = self.prefetch_count - len(self.unacked) if self.prefetch_count else 1 << 30
        if room <= 0:
            return 0
        for i, (qname, cb) in enumerate(self.consumers):
            q = self.broker.queues[qname]
            bulk = self.bulk.get(i)
            if bulk is None or not q.ready:
                continue
            pop, ready = q.ready.popleft, q.ready
            msgs = [pop() for _ in range(min(room, len(ready)))]
            t0 = next(self._tags)
            self._tags = itertools.count(t0 + len(msgs))
            tags = range(t0, t0 + len(msgs))
            self.unacked.update(zip(tags, msgs))
            bulk(self, tags, msgs)
            return len(msgs)
        return 0

    def start_consuming(self, until: Optional[Callable[[], bool]] = None) -> None:
        self.broker.run(until=until)

    def stop_consuming(self) -> None:
        self.broker.stop()

    def close(self) -> None:
        """Channel death: unacknowledged deliveries go back to their queues."""
        for tag in sorted(self.unacked, reverse=True):
            msg = self.unacked.pop(tag)
            msg.redelivered = True
            self.broker.queues[msg.queue].ready.appendleft(msg)
        self.is_open = False
        self.consumers = []


class MemoryBroker:
    """The broker and the ``BlockingConnection`` in one object."""

    def __init__(self, clock: Optional[Callable[[], float]] = None):
        self.clock = clock or time.monotonic
        self.queues: Dict[str, _Queue] = {}
        self.bindings: List[Tuple[str, str, "re.Pattern[str]"]] = []  # (exchange, queue, rx)
        self.channels: List[Channel] = []
        self.dropped: List[Message] = []        # routed nowhere
        self.dead_lettered: List[Message] = []  # nack(requeue=False)
        self.published: List[Message] = []     # every publish, in order (observability)
        self._timers: List[Tuple[float, int, Callable]] = []
        self._timer_ids = itertools.count(1)
        self._cancelled: set = set()
        self._stop = False

    # ----------------------------------------------------- connection surface
    def channel(self) -> Channel:
        ch = Channel(self, len(self.channels) + 1)
        self.channels.append(ch)
        return ch

    def add_timeout(self, deadline: float, callback: Callable[[], None]) -> int:
        tid = next(self._timer_ids)
        heapq.heappush(self._timers, (self.clock() + float(deadline), tid, callback))
        return tid

    def call_later(self, delay: float, callback: Callable[[], None]) -> int:  # pika >= 1.0 name
        return self.add_timeout(delay, callback)

    def remove_timeout(self, timeout_id: int) -> None:
        self._cancelled.add(timeout_id)

    def close(self) -> None:
        for ch in self.channels:
            if ch.is_open:
                ch.close()

    # --------------------------------------------------------------- routing
    def declare(self, queue: str, durable: bool = False) -> None:
        if queue not in self.queues:
            self.queues[queue] = _Queue(queue, durable)

    def bind(self, queue: str, exchange: str, routing_key: str) -> None:
        self.declare(queue)
        self.bindings.append((exchange, queue, _topic_regex(routing_key)))

    def publish(self, exchange: str, routing_key: str, body: bytes,
                properties: BasicProperties) -> None:
        msg = Message(body, properties, routing_key, exchange)
        self.published.append(msg)
        targets: List[str] = []
        if exchange == "":
            if routing_key in self.queues:
                targets = [routing_key]
        else:
            targets = [q for ex, q, rx in self.bindings if ex == exchange and rx.match(routing_key)]
        if not targets:
            self.dropped.append(msg)
            return
        for q in targets:
            self.queues[q].ready.append(Message(body, properties, routing_key, exchange, queue=q))

    def depth(self, queue: str) -> int:
        q = self.queues.get(queue)
        return len(q.ready) if q else 0

    def drain(self, queue: str) -> List[Message]:
        q = self.queues.get(queue)
        if not q:
            return []
        out = list(q.ready)
        q.ready.clear()
        return out

    # ------------------------------------------------------------ event loop
    def _fire_due_timers(self) -> bool:
        fired = False
        now = self.clock()
        while self._timers and self._timers[0][0] <= now:
            _, tid, cb = heapq.heappop(self._timers)
            if tid in self._cancelled:
                self._cancelled.discard(tid)
                continue
            cb()
            fired = True
        return fired

    def next_deadline(self) -> Optional[float]:
        while self._timers and self._timers[0][1] in self._cancelled:
            _, tid, _ = heapq.heappop(self._timers)
            self._cancelled.discard(tid)
        return self._timers[0][0] if self._timers else None

    def process_data_events(self, time_limit: float = 0.0) -> int:
        """Deliver everything deliverable now and fire due timers; returns the
        number of deliveries (``time_limit`` is accepted for pika compatibility)."""
        n = 0
        while True:
            progressed = self._fire_due_timers()
            for ch in self.channels:
                while True:
                    k = ch._deliver_bulk()
                    if not k:
                        if not ch._deliver_one():
                            break
                        k = 1
                    n += k
                    progressed = True
                    self._fire_due_timers()
            if not progressed:
                return n

    def run(self, until: Optional[Callable[[], bool]] = None, idle_exit: bool = True) -> None:
        """``start_consuming``: deliver and fire timers until ``stop()``, until
        ``until()`` is true, or -- with ``idle_exit`` -- until nothing is
        deliverable and no timer is pending.  A ManualClock jumps to the next
        timer; the real clock sleeps until it."""
        self._stop = False
        while not self._stop and not (until and until()):
            if self.process_data_events():
                continue
            dl = self.next_deadline()
            if dl is None:
                if idle_exit:
                    return
                time.sleep(0.01)
            elif isinstance(self.clock, ManualClock):
                self.clock.t = max(self.clock.t, dl)
            elif self.clock is time.monotonic:
                time.sleep(max(0.0, dl - self.clock()))
            else:
                return  # a custom clock that does not move by itself

    def stop(self) -> None:
        self._stop = True


class PikaChannel:
    """The worker's channel surface over a pika ``BlockingChannel``."""

    def __init__(self, pika, ch):
        self._pika = pika
        self._ch = ch
        # pika >= 1.0: basic_consume(queue, on_message_callback); 0.10: (callback, queue=)
        self._v1 = int(str(getattr(pika, "__version__", "0")).split(".")[0] or 0) >= 1

    def queue_declare(self, queue: str, durable: bool = False, **kw) -> None:
        self._ch.queue_declare(queue=queue, durable=durable, **kw)

    def basic_qos(self, prefetch_count: int = 0, **kw) -> None:
        self._ch.basic_qos(prefetch_count=int(prefetch_count), **kw)

    def basic_consume(self, *args, **kwargs) -> str:
        queue = kwargs.get("queue")
        callback = kwargs.get("on_message_callback") or kwargs.get("consumer_callback")
        for a in args:
            if callable(a):
                callback = a
            elif isinstance(a, str) and queue is None:
                queue = a
        if queue is None or callback is None:
            raise TypeError("basic_consume needs a queue and a callback")
        # pika hands (channel, method, properties, body) with the attribute names the
        # worker reads (method.delivery_tag, properties.headers); the worker acks
        # through this adapter, so give it the adapter as the channel
        cb = lambda _ch, method, props, body: callback(self, method, props, body)  # noqa: E731
        if self._v1:
            return self._ch.basic_consume(queue=queue, on_message_callback=cb)
        return self._ch.basic_consume(cb, queue=queue)

    def basic_ack(self, delivery_tag: int = 0, multiple: bool = False) -> None:
        self._ch.basic_ack(delivery_tag=delivery_tag, multiple=multiple)

    def basic_nack(self, delivery_tag: int = 0, multiple: bool = False, requeue: bool = True) -> None:
        self._ch.basic_nack(delivery_tag=delivery_tag, multiple=multiple, requeue=requeue)

    def basic_publish(self, exchange: str = "", routing_key: str = "", body=b"",
                      properties=None, **_) -> None:
        if isinstance(properties, BasicProperties):
            properties = self._pika.BasicProperties(headers=properties.headers,
                                                    delivery_mode=properties.delivery_mode,
                                                    content_type=properties.content_type)
        self._ch.basic_publish(exchange=exchange, routing_key=routing_key, body=body,
                               properties=properties)

    def close(self) -> None:
        self._ch.close()


class PikaBroker:
    """The worker's connection surface (``channel``, ``add_timeout`` /
    ``remove_timeout``, ``run``) over ``pika.BlockingConnection`` -- the
    reference's transport (/root/reference/worker.py:85-92,98-99,221)."""

    def __init__(self, uri: str, pika=None):
        if pika is None:
            import pika  # noqa: F811 -- optional dependency
        self._pika = pika
        self.conn = pika.BlockingConnection(pika.URLParameters(uri))
        self.channels: List[PikaChannel] = []
        self._stop = False

    def channel(self) -> PikaChannel:
        ch = PikaChannel(self._pika, self.conn.channel())
        self.channels.append(ch)
        return ch

    def add_timeout(self, delay: float, callback: Callable[[], None]):
        if hasattr(self.conn, "call_later"):   # pika >= 1.0
            return self.conn.call_later(delay, callback)
        return self.conn.add_timeout(delay, callback)  # pika 0.10

    def call_later(self, delay: float, callback: Callable[[], None]):
        return self.add_timeout(delay, callback)

    def remove_timeout(self, timeout_id) -> None:
        self.conn.remove_timeout(timeout_id)

    def process_data_events(self, time_limit: float = 0.0) -> None:
        self.conn.process_data_events(time_limit=time_limit)

    def run(self, until: Optional[Callable[[], bool]] = None, idle_exit: bool = False) -> None:
        """``start_consuming`` that also honours ``until`` / ``stop()``: the
        blocking loop in 0.1-s slices (deliveries and timers fire inside)."""
        self._stop = False
        while not self._stop and not (until and until()):
            self.conn.process_data_events(time_limit=0.1)

    def stop(self) -> None:
        self._stop = True

    def close(self) -> None:
        self.conn.close()


def connect(uri: str, clock: Optional[Callable[[], float]] = None):
    """Broker for a ``RABBITMQ_URI``.  ``memory://`` (or empty) -> in-process
    broker; ``tcp://host:port`` -> a ``BrokerServer`` that worker replicas share
    (runtime/broker_net.py); ``amqp://`` / ``amqps://`` -> ``PikaBroker`` (needs pika)."""
    if not uri or uri.startswith("memory:"):
        return MemoryBroker(clock)
    if uri.startswith("tcp://"):  # a BrokerServer shared by worker replicas (runtime/broker_net.py)
        from .broker_net import connect_tcp

        return connect_tcp(uri, clock)
    if uri.startswith("amqp"):
        try:
            import pika
        except ImportError as e:
            raise RuntimeError("RABBITMQ_URI=%s needs the pika package, which is not installed; "
                               "use RABBITMQ_URI=memory:// for the in-process broker" % uri) from e
        return PikaBroker(uri, pika)
    raise ValueError("unsupported broker URI %r" % uri)
