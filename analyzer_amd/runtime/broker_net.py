"""A broker process that several worker replicas share over TCP: ``tcp://host:port``
(SURVEY P1 "replica scale-out"; WHAT's missing #4 of the round-4 verdict).

The reference scales horizontally by running N worker processes on one RabbitMQ queue
with a prefetch of ``BATCHSIZE`` each (/root/reference/worker.py:91).  With RabbitMQ the
same works here through the pika adapter (``amqp://``, runtime/broker.py).  This image
has no RabbitMQ, so ``BrokerServer`` hosts the in-process ``MemoryBroker`` -- the same
AMQP 0-9-1 semantics: per-consumer prefetch windows, redelivery of a dead consumer's
unacknowledged messages, the default and topic exchanges -- behind a small TCP protocol,
and ``NetBroker`` is the worker's connection surface over it (``channel``,
``add_timeout`` / ``remove_timeout``, ``run``).  ``worker.py --replicas N`` starts one
server and N worker processes, one per GPU (runtime/replicas.py).

Wire format: frames of a 4-byte big-endian length and a msgpack list.  Requests carry a
sequence number and get a ``reply``; publishes, acks and nacks are one-way.  The server
pushes ``deliver`` frames to each connection's consumer as prefetch credit allows (one
message at a time, round-robin over the connected consumers, as RabbitMQ does).
"""
from __future__ import annotations

import heapq
import itertools
import queue as _queue
import select
import socket
import struct
import threading
import time
from collections import deque
from typing import Callable, Deque, Dict, List, Optional, Tuple

import msgpack

from .broker import BasicProperties, MemoryBroker, Method

_HDR = struct.Struct(">I")


def _pack(frame) -> bytes:
    body = msgpack.packb(frame, use_bin_type=True)
    return _HDR.pack(len(body)) + body


def _props(headers, mode, ctype) -> BasicProperties:
    return BasicProperties(headers=headers, delivery_mode=mode, content_type=ctype)


class _FrameReader:
    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes) -> List[list]:
        self.buf += data
        out = []
        while len(self.buf) >= 4:
            (n,) = _HDR.unpack_from(self.buf, 0)
            if len(self.buf) < 4 + n:
                break
            out.append(msgpack.unpackb(bytes(self.buf[4:4 + n]), raw=False))
            del self.buf[:4 + n]
        return out


# --------------------------------------------------------------------------- server
class _ServerConn:
    """One client connection: a server-side channel of the shared MemoryBroker, a
    reader thread applying its frames and a writer thread draining its outbox."""

    def __init__(self, server: "BrokerServer", sock: socket.socket):
        self.server = server
        self.sock = sock
        self.out: "_queue.Queue[Optional[bytes]]" = _queue.Queue()
        with server.lock:
            self.ch = server.broker.channel()
        self.alive = True

    def start(self) -> None:
        threading.Thread(target=self._reader, daemon=True).start()
        threading.Thread(target=self._writer, daemon=True).start()

    def _deliver(self, _ch, method: Method, props: BasicProperties, body: bytes) -> None:
        # called under the server lock from MemoryBroker delivery: queue the frame only
        self.out.put(_pack(["deliver", method.delivery_tag, method.routing_key, method.exchange,
                            method.redelivered, body, props.headers, props.delivery_mode, props.content_type]))

    def _writer(self) -> None:
        while True:
            data = self.out.get()
            if data is None:
                return
            try:
                self.sock.sendall(data)
            except OSError:
                return

    def _apply(self, f: list):
        op = f[0]
        ch, b = self.ch, self.server.broker
        if op == "publish":
            _, ex, key, body, headers, mode, ctype = f
            b.publish(ex, key, bytes(body), _props(headers, mode, ctype))
        elif op == "ack":
            ch.basic_ack(f[1], multiple=f[2])
        elif op == "nack":
            ch.basic_nack(f[1], multiple=f[2], requeue=f[3])
        elif op == "declare":
            b.declare(f[2], f[3])
        elif op == "bind":
            b.bind(f[2], f[3], f[4])
        elif op == "qos":
            ch.basic_qos(prefetch_count=f[2])
        elif op == "consume":
            return ch.basic_consume(self._deliver, queue=f[2])
        elif op == "depth":
            return b.depth(f[2])
        elif op == "in_flight":
            return self.server.in_flight(f[2])
        elif op == "stats":
            return self.server.stats()
        else:
            raise ValueError("unknown broker op %r" % op)
        return None

    def _reader(self) -> None:
        rd = _FrameReader()
        try:
            while True:
                data = self.sock.recv(1 << 16)
                if not data:
                    break
                for f in rd.feed(data):
                    with self.server.lock:
                        try:
                            res, err = self._apply(f), None
                        except Exception as e:  # reported to a request, else dropped with the connection
                            res, err = None, "%s: %s" % (type(e).__name__, e)
                        if f[0] in ("declare", "bind", "qos", "consume", "depth", "in_flight", "stats"):
                            self.out.put(_pack(["reply", f[1], res, err]))
                        elif err is not None:
                            raise RuntimeError(err)
                    self.server.pump()
        except (OSError, RuntimeError):
            pass
        finally:
            self.close()

    def close(self) -> None:
        if not self.alive:
            return
        self.alive = False
        with self.server.lock:
            self.ch.close()  # consumer death: its unacknowledged deliveries are requeued
            self.server.conns.discard(self)
        self.out.put(None)
        try:
            self.sock.close()
        except OSError:
            pass
        self.server.pump()


class BrokerServer:
    """The shared broker: ``BrokerServer(port=0).start()``; ``uri`` names it."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.broker = MemoryBroker()
        self.lock = threading.RLock()
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.host, self.port = self.sock.getsockname()[:2]
        self.conns: set = set()
        self._closed = False

    @property
    def uri(self) -> str:
        return "tcp://%s:%d" % (self.host, self.port)

    def start(self) -> "BrokerServer":
        threading.Thread(target=self._accept, daemon=True).start()
        return self

    def _accept(self) -> None:
        while not self._closed:
            try:
                s, _ = self.sock.accept()
            except OSError:
                return
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = _ServerConn(self, s)
            with self.lock:
                self.conns.add(c)
            c.start()

    def pump(self) -> int:
        """Deliver what prefetch credit allows, one message per channel per round
        (round-robin over the consumers, as RabbitMQ dispatches)."""
        n = 0
        with self.lock:
            progressed = True
            while progressed:
                progressed = False
                for ch in list(self.broker.channels):
                    if ch.is_open and ch._deliver_one():
                        n += 1
                        progressed = True
        return n

    def publish(self, queue: str, bodies, durable: bool = True) -> None:
        """Declare ``queue`` and enqueue ``bodies`` on the default exchange (a producer
        in the server's own process: runtime/replicas.py)."""
        with self.lock:
            self.broker.declare(queue, durable)
            for b in bodies:
                self.broker.publish("", queue, b if isinstance(b, bytes) else str(b).encode(), BasicProperties())
        self.pump()

    def in_flight(self, queue: str) -> int:
        """Messages of ``queue`` not yet settled anywhere: ready ones plus every open
        consumer's unacknowledged deliveries.  A replica may only leave when this is
        zero -- if another replica still holds a prefetch window and dies, its
        deliveries are requeued and need a consumer (at-least-once)."""
        with self.lock:
            b = self.broker
            held = sum(1 for c in b.channels if c.is_open for m in c.unacked.values() if m.queue == queue)
            return b.depth(queue) + held

    def stats(self) -> Dict[str, object]:
        with self.lock:
            b = self.broker
            return {"depth": {q: len(v.ready) for q, v in b.queues.items()},
                    "acked": sum(c.acked for c in b.channels), "nacked": sum(c.nacked for c in b.channels),
                    "dead_lettered": len(b.dead_lettered), "dropped": len(b.dropped),
                    "unacked": sum(len(c.unacked) for c in b.channels if c.is_open),
                    "consumers": sum(1 for c in b.channels if c.is_open and c.consumers)}

    def close(self) -> None:
        self._closed = True
        try:
            self.sock.close()
        except OSError:
            pass
        for c in list(self.conns):
            c.close()


# --------------------------------------------------------------------------- client
class NetChannel:
    """The worker's channel surface (runtime/broker.py Channel) over a NetBroker."""

    def __init__(self, conn: "NetBroker"):
        self.conn = conn
        self.consumers: List[Tuple[str, Callable]] = []
        self.outstanding: set = set()  # delivered, not yet settled (this client's view)
        self.is_open = True

    def queue_declare(self, queue: str, durable: bool = False, **_) -> None:
        self.conn._request("declare", queue, bool(durable))

    def queue_bind(self, queue: str, exchange: str, routing_key: str) -> None:
        self.conn._request("bind", queue, exchange, routing_key)

    def basic_qos(self, prefetch_count: int = 0, **_) -> None:
        self.conn._request("qos", int(prefetch_count))

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
        if self.consumers:
            raise RuntimeError("NetChannel: one consumer per connection")
        self.consumers.append((queue, callback))
        return self.conn._request("consume", queue)

    def basic_publish(self, exchange: str = "", routing_key: str = "", body=b"",
                      properties: Optional[BasicProperties] = None, **_) -> None:
        if isinstance(body, str):
            body = body.encode("utf-8")
        p = properties or BasicProperties()
        self.conn._send(["publish", exchange, routing_key, bytes(body), p.headers, p.delivery_mode,
                         p.content_type])

    def _settle(self, tag: int, multiple: bool) -> None:
        if multiple:
            self.outstanding = {t for t in self.outstanding if t > tag} if tag else set()
        else:
            self.outstanding.discard(tag)

    def basic_ack(self, delivery_tag: int = 0, multiple: bool = False) -> None:
        self._settle(delivery_tag, multiple)
        self.conn._send(["ack", int(delivery_tag), bool(multiple)])

    def basic_nack(self, delivery_tag: int = 0, multiple: bool = False, requeue: bool = True) -> None:
        self._settle(delivery_tag, multiple)
        self.conn._send(["nack", int(delivery_tag), bool(multiple), bool(requeue)])

    def basic_reject(self, delivery_tag: int, requeue: bool = True) -> None:
        self.basic_nack(delivery_tag, requeue=requeue)

    def start_consuming(self, until: Optional[Callable[[], bool]] = None) -> None:
        self.conn.run(until=until)

    def stop_consuming(self) -> None:
        self.conn.stop()

    def close(self) -> None:
        self.is_open = False
        self.conn.close()


class NetBroker:
    """The worker's connection surface over a BrokerServer: ``connect("tcp://h:p")``.

    ``run`` delivers and fires timers until ``stop()`` / ``until()``; with ``idle_exit``
    (default) it also returns once nothing is in flight here, no timer is pending and
    the server reports nothing of the consumed queue unsettled -- neither ready nor held
    unacknowledged by another replica (which could still die and have its window
    requeued) -- so the last replica leaves only when the queue is truly drained."""

    def __init__(self, host: str, port: int, clock: Optional[Callable[[], float]] = None):
        self.clock = clock or time.monotonic
        self.sock = socket.create_connection((host, port))
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._rd = _FrameReader()
        self._deliveries: Deque[list] = deque()
        self._replies: Dict[int, list] = {}
        self._seq = itertools.count(1)
        self._timers: List[Tuple[float, int, Callable]] = []
        self._timer_ids = itertools.count(1)
        self._cancelled: set = set()
        self._ch: Optional[NetChannel] = None
        self._stop = False
        self.closed = False

    # -------------------------------------------------------------- transport
    def _send(self, frame) -> None:
        self.sock.sendall(_pack(frame))

    def _read(self, timeout: float) -> bool:
        r, _, _ = select.select([self.sock], [], [], max(0.0, timeout))
        if not r:
            return False
        data = self.sock.recv(1 << 16)
        if not data:
            raise ConnectionError("broker closed the connection")
        for f in self._rd.feed(data):
            if f[0] == "deliver":
                self._deliveries.append(f)
            elif f[0] == "reply":
                self._replies[f[1]] = f
        return True

    def _request(self, op: str, *args):
        seq = next(self._seq)
        self._send([op, seq, *args])
        while seq not in self._replies:
            self._read(1.0)
        _, _, res, err = self._replies.pop(seq)
        if err:
            raise RuntimeError("broker: %s" % err)
        return res

    # -------------------------------------------------------- connection surface
    def channel(self) -> NetChannel:
        if self._ch is not None:
            raise RuntimeError("NetBroker: one channel per connection")
        self._ch = NetChannel(self)
        return self._ch

    def add_timeout(self, deadline: float, callback: Callable[[], None]) -> int:
        tid = next(self._timer_ids)
        heapq.heappush(self._timers, (self.clock() + float(deadline), tid, callback))
        return tid

    def call_later(self, delay: float, callback: Callable[[], None]) -> int:
        return self.add_timeout(delay, callback)

    def remove_timeout(self, timeout_id: int) -> None:
        self._cancelled.add(timeout_id)

    def next_deadline(self) -> Optional[float]:
        while self._timers and self._timers[0][1] in self._cancelled:
            _, tid, _ = heapq.heappop(self._timers)
            self._cancelled.discard(tid)
        return self._timers[0][0] if self._timers else None

    def depth(self, queue: str) -> int:
        return int(self._request("depth", queue))

    def in_flight(self, queue: str) -> int:
        """Ready + unacknowledged-anywhere messages of ``queue`` (BrokerServer.in_flight)."""
        return int(self._request("in_flight", queue))

    def stats(self) -> Dict[str, object]:
        return self._request("stats")

    # ---------------------------------------------------------------- event loop
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

    def _dispatch(self) -> int:
        n = 0
        ch = self._ch
        while self._deliveries:
            _, tag, key, ex, redelivered, body, headers, mode, ctype = self._deliveries.popleft()
            if ch is None or not ch.consumers:
                continue
            ch.outstanding.add(tag)
            ch.consumers[0][1](ch, Method(tag, key, ex, redelivered), _props(headers, mode, ctype), bytes(body))
            n += 1
            self._fire_due_timers()
        return n

    def process_data_events(self, time_limit: float = 0.0) -> int:
        fired = self._fire_due_timers()
        while self._read(0.0):
            pass
        return self._dispatch() + int(fired)

    def run(self, until: Optional[Callable[[], bool]] = None, idle_exit: bool = True) -> None:
        self._stop = False
        queue = self._ch.consumers[0][0] if self._ch is not None and self._ch.consumers else None
        while not self._stop and not (until and until()):
            if self.process_data_events():
                continue
            dl = self.next_deadline()
            wait = 0.05 if dl is None else min(0.05, max(0.0, dl - self.clock()))
            if self._read(wait):
                continue
            if (idle_exit and dl is None and queue is not None and not self._ch.outstanding
                    and not self._deliveries and self.in_flight(queue) == 0):
                # nothing here or in the queue; a last look for deliveries sent meanwhile
                if not self._read(0.05) and not self._deliveries:
                    return

    def stop(self) -> None:
        self._stop = True

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass


def connect_tcp(uri: str, clock: Optional[Callable[[], float]] = None) -> NetBroker:
    hostport = uri[len("tcp://"):].rstrip("/")
    host, _, port = hostport.rpartition(":")
    return NetBroker(host or "127.0.0.1", int(port), clock)
