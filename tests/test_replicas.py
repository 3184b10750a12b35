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


def test_idle_exit_waits_for_other_replicas_unacked_windows():
    """A consumer with nothing of its own in flight must not leave while another
    consumer still holds unacknowledged deliveries: if that one dies, its window is
    requeued and needs a consumer (at-least-once; BrokerServer.in_flight)."""
    srv = BrokerServer().start()
    try:
        srv.publish("q", [b"m%d" % i for i in range(4)])
        a = connect(srv.uri)
        ca = a.channel()
        ca.basic_qos(prefetch_count=10)
        held = []
        ca.basic_consume(lambda ch, m, p, body: held.append(m.delivery_tag), queue="q")
        while len(held) < 4:
            a._read(0.05)
            a.process_data_events()
        assert srv.in_flight("q") == 4 and srv.stats()["depth"]["q"] == 0
        b = connect(srv.uri)
        cb = b.channel()
        cb.basic_qos(prefetch_count=10)
        got = []

        def on(ch, m, p, body):
            got.append(body)
            ch.basic_ack(m.delivery_tag)
        cb.basic_consume(on, queue="q")
        t = threading.Thread(target=b.run)
        t.start()
        t.join(0.5)
        assert t.is_alive()  # the queue is empty, but a's window is not settled
        a.close()            # a dies holding 4 deliveries: they go to b
        t.join(10.0)
        assert not t.is_alive() and len(got) == 4
        assert srv.in_flight("q") == 0
        b.close()
    finally:
        srv.close()


def test_visible_device_mapping_follows_the_parent():
    from analyzer_amd.runtime.replicas import _visible_devices

    assert _visible_devices({"HIP_VISIBLE_DEVICES": "4,5"}, 2) == ["4", "5"]
    assert _visible_devices({}, 3) == ["0", "1", "2"]
    assert _visible_devices({"ROCR_VISIBLE_DEVICES": "6,7"}, 2) == ["0", "1"]


def _player_rows(path):
    from analyzer_amd.runtime.store import PLAYER_RATING_COLS, _q

    con = sqlite3.connect(path)
    rows = con.execute("SELECT api_id, %s FROM player ORDER BY api_id"
                       % ", ".join(_q(c) for c in PLAYER_RATING_COLS)).fetchall()
    con.close()
    return rows


def _replay(path_log, path_fresh, n_matches, n_players, seed, engine):
    """Rate the logged batches one after another, in commit order, with one in-process
    worker on a fresh copy of the initial store."""
    from analyzer_amd.config import WorkerConfig
    from analyzer_amd.runtime.broker import MemoryBroker
    from analyzer_amd.runtime.source import populate
    from analyzer_amd.runtime.store import SqliteStore
    from analyzer_amd.runtime.worker import Worker

    con = sqlite3.connect(path_log)
    log = [r[0].split(",") for r in con.execute("SELECT match_ids FROM batch_log ORDER BY seq")]
    con.close()
    store = SqliteStore(path_fresh)
    populate(store, n_matches, n_players, seed=seed)
    w = Worker(WorkerConfig(engine=engine, resident=False, rabbitmq_uri="memory://"), store=store,
               broker=MemoryBroker())
    w.connect()
    for ids in log:
        w.process([(None, None, i.encode()) for i in ids])
    store.close()
    return log


@pytest.mark.parametrize("engine", ["native", "python"])
def test_replicas_lose_no_update(tmp_path, engine):
    """Four replicas over matches that share players (60 players, 600 3v3 matches,
    batches of 20): every player write is a compare-and-set on the row version, and a
    batch that lost the race is rated again -- so the final ratings equal rating the
    committed batches one after another in commit order (the BATCH_LOG replay), i.e.
    no replica's update was overwritten.  The reference's replicas race on exactly these
    rows (/root/reference/worker.py:174-194)."""
    n, players, seed = 600, 60, 13
    env = dict(os.environ, ENGINE=engine, BATCHSIZE="20", IDLE_TIMEOUT="0.05", BATCH_LOG="true")
    db = str(tmp_path / "r.db")
    res = run_replicas(4, synthetic=n, players=players, seed=seed, env=env, database_uri="sqlite:///" + db)
    assert res["ok"] and res["exit_codes"] == [0, 0, 0, 0], res
    assert res["acked"] == n and res["unsettled"] == 0
    log = _replay(db, str(tmp_path / "replay.db"), n, players, seed, engine)
    assert sorted(i for b in log for i in b) == sorted(set(i for b in log for i in b))  # each match once
    assert len([i for b in log for i in b]) == n
    assert _player_rows(db) == _player_rows(str(tmp_path / "replay.db"))
