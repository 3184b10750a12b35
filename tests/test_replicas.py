"""Horizontal scale-out of the streaming worker (runtime/replicas.py, broker_net.py):
N worker processes on one queue of a shared broker and one SQLite store, as the
reference runs N replicas on RabbitMQ + MySQL (/root/reference/worker.py:91)."""
import os
import sqlite3
import threading

import pytest

from analyzer_amd.runtime.broker import connect
from analyzer_amd.runtime.broker_net import BrokerServer
from analyzer_amd.runtime.replicas import run_replicas


def test_tcp_broker_prefetch_ack_and_redelivery():
    """Prefetch windows per consumer, acks, and a dead consumer's unacknowledged
    deliveries going to the next consumer (redelivered=True), over the TCP protocol."""
    srv = BrokerServer().start()
    try:
        srv.publish("q", [b"m%d" % i for i in range(10)])
        a = connect(srv.uri)
        ca = a.channel()
        ca.queue_declare("q", durable=True)
        ca.basic_qos(prefetch_count=3)
        held = []
        ca.basic_consume(lambda ch, m, p, body: held.append((m.delivery_tag, body)), queue="q")
        while len(held) < 3:
            a.process_data_events()
            a._read(0.05)
        a.process_data_events()
        assert len(held) == 3  # the prefetch window, nothing more while unacked
        ca.basic_ack(held[0][0])
        while len(held) < 4:
            a._read(0.05)
            a.process_data_events()
        a.close()  # dies holding 3 unacked deliveries
        b = connect(srv.uri)
        cb = b.channel()
        cb.basic_qos(prefetch_count=100)
        got = []

        def on(ch, m, p, body):
            got.append((body, m.redelivered))
            ch.basic_ack(m.delivery_tag)
        cb.basic_consume(on, queue="q")
        b.run()
        bodies = [g[0] for g in got]
        assert sorted(bodies + [held[0][1]]) == sorted(b"m%d" % i for i in range(10))
        assert sum(r for _, r in got) == 3  # the dead consumer's deliveries come back flagged
        st = srv.stats()
        assert st["depth"]["q"] == 0 and st["acked"] == 10 and st["unacked"] == 0
        b.close()
    finally:
        srv.close()


def _rated(uri):
    con = sqlite3.connect(uri[len("sqlite:///"):])
    n = con.execute("SELECT count(*) FROM match WHERE trueskill_quality IS NOT NULL").fetchone()[0]
    tot = con.execute("SELECT count(*) FROM match").fetchone()[0]
    con.close()
    return n, tot


@pytest.mark.parametrize("engine", ["native", "python"])
def test_replicas_drain_one_queue(tmp_path, engine):
    """Three worker processes share the queue and the store file: every message is
    acked once and every match is rated once (how the work spreads depends on start-up
    order; the replica-death test below makes the others take over a share)."""
    env = dict(os.environ, ENGINE=engine, BATCHSIZE="40", IDLE_TIMEOUT="0.2")
    res = run_replicas(3, synthetic=600, seed=5, env=env, database_uri="sqlite:///%s" % (tmp_path / "s.db"))
    assert res["exit_codes"] == [0, 0, 0], res
    assert res["matches"] == 600 and res["acked"] == 600 and res["nacked"] == 0
    assert res["broker"]["depth"][next(iter(res["broker"]["depth"]))] == 0
    assert res["broker"]["acked"] == 600 and res["broker"]["unacked"] == 0
    assert sum(int(r["matches"] or 0) for r in res["per_replica"]) == 600  # each message rated once
    n, tot = _rated(res["database_uri"])
    assert tot == 600 and n >= 550  # AFK / invalid matches keep no quality


def test_replica_death_redelivers_to_the_others(tmp_path):
    """Replica 0 dies (exit 17) holding a batch of unacked deliveries after one
    batch: the broker redelivers them, the other replicas rate them, and the store
    ends with every match rated -- at-least-once, as with RabbitMQ."""
    env = dict(os.environ, ENGINE="native", BATCHSIZE="40", IDLE_TIMEOUT="0.2")
    res = run_replicas(3, synthetic=600, seed=6, env=env, database_uri="sqlite:///%s" % (tmp_path / "d.db"),
                       replica_env={0: {"FAULT_EXIT_AFTER": "1"}}, first_alone_until_acked=40)
    assert res["exit_codes"][0] == 17 and res["exit_codes"][1:] == [0, 0], res
    assert res["broker"]["acked"] == 600 and res["broker"]["unacked"] == 0
    assert res["broker"]["dead_lettered"] == 0
    n_single = _rated(res["database_uri"])
    assert n_single[1] == 600 and n_single[0] >= 550
