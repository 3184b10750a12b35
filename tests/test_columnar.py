"""Columnar worker path (runtime/columnar.py + runtime/resident.py rate_batch):
ColumnarStore and SQLite batches rated against the resident roster give what the
reference-semantics Python engine writes, transactions roll back on the device
too, and telemetry lands in the columns.  CPU (host mirror) -- the GPU run of the
same path is scripts/gpu.sh worker."""
import math

import numpy as np
import pytest

from analyzer_amd.config import RaterConfig, WorkerConfig
from analyzer_amd.runtime import broker as B
from analyzer_amd.runtime.columnar import ColumnarStore
from analyzer_amd.runtime.source import populate, publish
from analyzer_amd.runtime.store import MemoryStore, open_store
from analyzer_amd.runtime.worker import Worker

TRACKS = ("trueskill", "trueskill_casual", "trueskill_ranked", "trueskill_blitz", "trueskill_br")


def run(store, engine, n=60, players=25, batch=16, seed=7, quarantine=True, before=None, **flags):
    clock = B.ManualClock()
    cfg = WorkerConfig(batchsize=batch, chunksize=5, idle_timeout=1.0, engine=engine,
                       quarantine=quarantine, **flags)
    ms = populate(store, n, players, team_size=3, seed=seed)
    ids = [m.api_id for m in ms]
    if before is not None:
        before(store)
    w = Worker(cfg, store=store, broker=B.MemoryBroker(clock), rater_cfg=RaterConfig(), clock=clock)
    w.connect()
    publish(w.channel, "analyze", ids)
    w.start_consuming()
    return w, ids


def snapshot(store, ids):
    """Everything the rater writes, read back through a fresh session."""
    out = {}
    s = store.session()
    for m in s.load_matches(ids):
        out[m.api_id] = ("q", m.trueskill_quality)
        for p in m.participants:
            it = p.participant_items[0]
            out[p.api_id] = (p.trueskill_mu, p.trueskill_sigma, p.trueskill_delta, it.any_afk) + tuple(
                getattr(it, c + s_) for c in TRACKS[1:] for s_ in ("_mu", "_sigma"))
            pl = p.player[0]
            out["player:" + pl.api_id] = tuple(getattr(pl, c + s_) for c in TRACKS for s_ in ("_mu", "_sigma"))
    s.close()
    return out


def assert_same(a, b, tol):
    assert a.keys() == b.keys()
    for k in a:
        for x, y in zip(a[k], b[k]):
            if isinstance(x, str):
                continue
            assert (x is None) == (y is None), (k, a[k], b[k])
            if x is not None:
                assert abs(float(x) - float(y)) <= tol, (k, a[k], b[k])


def test_columnar_native_matches_python_engine_on_object_store():
    wr, ids = run(MemoryStore(), "python")
    ref = snapshot(wr.store, ids)
    col = ColumnarStore()
    wc, ids_c = run(col, "native")
    assert ids_c == ids and wc.stats.matches == 60 and wc.stats.acked == 60
    assert_same(snapshot(col, ids), ref, 2e-3)  # fp32 state (host mirror fp64 arithmetic)


def test_columnar_object_path_is_the_python_engine_exactly():
    wr, ids = run(MemoryStore(), "python")
    col = ColumnarStore()
    run(col, "python")
    assert_same(snapshot(col, ids), snapshot(wr.store, ids), 0.0)


def test_sqlite_batches_match_python_engine(tmp_path):
    a = open_store("sqlite:///" + str(tmp_path / "a.db"))
    b = open_store("sqlite:///" + str(tmp_path / "b.db"))
    _, ids = run(a, "python")
    wb, _ = run(b, "native")
    assert wb.stats.acked == 60
    assert_same(snapshot(b, ids), snapshot(a, ids), 2e-3)


def _poison(store):
    """One player without a rating and with tier 30: the reference raises KeyError."""
    if isinstance(store, ColumnarStore):
        r = store.pl_index["p3"]
        store.players.rating[r] = np.nan
        store.players.attr[r] = [np.nan, np.nan, 30.0]
    else:
        pl = store.players["p3"]
        pl.trueskill_mu = pl.trueskill_sigma = None
        for c in TRACKS[1:]:
            setattr(pl, c + "_mu", None)
            setattr(pl, c + "_sigma", None)
        pl.rank_points_ranked = pl.rank_points_blitz = None
        pl.skill_tier = 30


@pytest.mark.parametrize("quarantine", [True, False])
def test_columnar_failures_match_python_engine(quarantine):
    """QUARANTINE=true: only the poisoned player's matches go to <queue>_failed.
    QUARANTINE=false: each batch holding one fails whole and is rolled back --
    on the device roster too, so later batches rate from the committed state
    exactly like the Python engine."""
    wr, ids = run(MemoryStore(), "python", quarantine=quarantine, before=_poison)
    col = ColumnarStore()
    wc, _ = run(col, "native", quarantine=quarantine, before=_poison)
    failed_r = sorted(m.body for m in wr.rabbit.drain("analyze_failed"))
    failed_c = sorted(m.body for m in wc.rabbit.drain("analyze_failed"))
    assert failed_c == failed_r and len(failed_r) > 0
    assert wc.stats.failed_batches == wr.stats.failed_batches
    assert (wc.stats.failed_batches > 0) == (not quarantine)
    assert_same(snapshot(col, ids), snapshot(wr.store, ids), 2e-3)


def test_columnar_telemetry_into_participant_stats():
    col = ColumnarStore()
    w, ids = run(col, "native", n=10, players=20, batch=10, dotelemetry=True, telemetry_events="5,9")
    assert w.stats.acked == 10
    s = col.session()
    total = 0.0
    for m in s.load_matches(ids):
        for p in m.participants:
            st = s.participant_stats(p.api_id)
            assert st is not None and st["events"] >= 0
            total += st["events"]
    assert 5 * 10 <= total <= 9 * 10


def test_resident_roster_failed_fetch_leaves_no_rows():
    """A fetch that raises (store error) must not map keys to unwritten rows."""
    from analyzer_amd.runtime.resident import ResidentRoster

    rr = ResidentRoster("cpu", capacity=4)

    def boom(keys):
        raise IOError("store down")

    with pytest.raises(IOError):
        rr.rows_for_keys(np.array([3, 7]), boom)
    assert rr.n == 0 and (rr.by_key < 0).all()
    ok = lambda keys: (np.full((len(keys), 14), np.nan), np.zeros((len(keys), 3)))
    assert rr.rows_for_keys(np.array([7, 3]), ok).tolist() == [0, 1]
    assert rr.rows_for_keys(np.array([3, 9]), ok).tolist() == [1, 2]


def _mixed_store(seed=3, n=40, players=30):
    """Matches of 1-3 rosters, uneven sizes, AFKs (also in a third roster),
    unsupported modes, ties in created_at."""
    from analyzer_amd.runtime.objects import Match, Participant, Player, Roster

    rng = np.random.default_rng(seed)
    pl = [Player("q%d" % i, int(rng.integers(1, 30)), None, None,
                 trueskill_mu=float(rng.normal(25, 3)), trueskill_sigma=float(rng.uniform(2, 8)))
          for i in range(players)]
    col = ColumnarStore()
    ms = []
    for i in range(n):
        nr = int(rng.choice([1, 2, 2, 2, 3]))
        rosters = []
        for ri in range(nr):
            k = int(rng.integers(1, 4))
            ps = [Participant(pl[int(rng.integers(players))], "m%dr%dp%d" % (i, ri, j),
                              went_afk=int(rng.random() < 0.1)) for j in range(k)]
            rosters.append(Roster(ps, winner=bool(ri == 0) if rng.random() < 0.9 else None,
                                  api_id="m%dr%d" % (i, ri)))
        mode = str(rng.choice(["casual", "ranked", "blitz", "5v5_casual", "private"]))
        ms.append(Match(mode, rosters, api_id="m%d" % i, created_at=float(i // 3)))
    col.add_matches(ms)
    return col, [m.api_id for m in ms]


def test_native_batch_gather_matches_numpy():
    col, ids = _mixed_store()
    s = col.session()
    a, b = s.load_batch(ids), s._load_batch_numpy(ids)
    assert a.ids == b.ids and a.extra_parts == b.extra_parts and a.K == b.K
    for f in ("mode", "nrosters", "n", "winner", "afk", "player", "part", "rows"):
        x, y = getattr(a, f), getattr(b, f)
        assert x.shape == y.shape and (np.asarray(x, np.int64) == np.asarray(y, np.int64)).all(), f
    assert any(len(v) for v in a.extra_parts.values())


def test_native_batch_commit_matches_numpy():
    """rate_batch (native encode / finish) then batch_commit writes exactly what
    the numpy finish + _write_batch_numpy write, extra rosters included."""
    import copy

    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.runtime.resident import ResidentBatchRater

    col, ids = _mixed_store(seed=5)
    twin = copy.deepcopy(col)
    rb = ResidentBatchRater(BatchRater(RaterConfig()), device="cpu", capacity=64)
    s = col.session()
    mb = s.load_batch(ids)
    rb.rate_batch(mb, s.fetch_players)
    assert (mb.status == 0).any() and (mb.status == 1).any()
    s.commit()
    t = twin.session()
    mb2 = t._load_batch_numpy(ids)
    for f in ("status", "quality", "s_mu", "s_sig", "delta", "m_mu", "m_sig", "final_keys", "final",
              "final_tracks"):
        setattr(mb2, f, getattr(mb, f))
    t._write_batch_numpy(mb2)
    for tab, cols in (("matches", ("quality",)), ("parts", ("i_afk", "ts", "i_rating")), ("players", ("rating",))):
        for c in cols:
            x, y = getattr(getattr(col, tab), c), getattr(getattr(twin, tab), c)
            assert np.array_equal(x, y, equal_nan=True), (tab, c)


def test_rate_batch_failed_fetch_leaves_no_rows():
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.runtime.resident import ResidentBatchRater

    col, ids = _mixed_store(seed=9, n=10)
    rb = ResidentBatchRater(BatchRater(RaterConfig()), device="cpu", capacity=16)
    s = col.session()
    mb = s.load_batch(ids)

    def boom(keys):
        raise IOError("store down")

    with pytest.raises(IOError):
        rb.rate_batch(mb, boom)
    assert rb.resident.n == 0 and (rb.resident.by_key < 0).all()
    rb.rate_batch(mb, s.fetch_players)
    assert rb.resident.n == len(np.unique(mb.player[mb.player >= 0]))


def test_native_player_staging_matches_upload_arrays():
    from analyzer_amd.runtime.resident import ResidentRoster

    col, _ = _mixed_store(seed=4, players=50)
    rng = np.random.default_rng(0)
    col.players.rating[:50][rng.random((50, 14)) < 0.3] = np.nan  # NULL tracks and NULL sigmas
    keys = np.array([7, 3, 41, 0, 19], dtype=np.int64)
    a, b = ResidentRoster("cpu", 4), ResidentRoster("cpu", 4)
    a._upload_arrays(*col.session().fetch_players(keys))
    buf = b.staging(len(keys))
    col.session().stage_players(__import__("torch").from_numpy(keys), buf)
    b.upload_staged(buf)
    assert np.array_equal(a.roster.state.numpy(), b.roster.state.numpy(), equal_nan=True)
    assert np.array_equal(a.roster.attrs.numpy(), b.roster.attrs.numpy(), equal_nan=True)


def test_native_key_index():
    from analyzer_amd.ops.native import native

    ki = native().KeyIndex()
    keys = ["m%d" % i for i in range(5000)] + ["é-%d" % i for i in range(100)]
    ki.add(keys[:3000], 0)
    ki.add(keys[3000:], 3000)  # grows the table
    assert len(ki) == len(keys)
    q = ["m17", b"m4999", "nope", "é-7".encode(), "é-99", "m0", b""]
    assert ki.lookup(q).tolist() == [17, 4999, -1, 5007, 5099, 0, -1]
    with pytest.raises(ValueError):
        ki.add(["m5"], 9)
    col, ids = _mixed_store()
    rows = col.match_rows(ids[::-1] + ["missing"])
    assert rows.tolist() == [col.m_index[i] for i in ids[::-1]] + [-1]


@pytest.mark.parametrize("quarantine", [True, False])
def test_fault_injection_poison_matches_python_engine(quarantine):
    """FAULT_POISON: the named matches fail in both engines -- the same failed
    queue, failed batches and store contents (SURVEY §5 fault injection)."""
    poison = frozenset({"m3", "m17", "m40"})
    wr, ids = run(MemoryStore(), "python", quarantine=quarantine, fault_poison=poison)
    col = ColumnarStore()
    wc, _ = run(col, "native", quarantine=quarantine, fault_poison=poison)
    failed_r = sorted(m.body for m in wr.rabbit.drain("analyze_failed"))
    failed_c = sorted(m.body for m in wc.rabbit.drain("analyze_failed"))
    assert failed_c == failed_r
    if quarantine:
        assert sorted(failed_r) == sorted(x.encode() for x in poison)
    assert wc.stats.failed_batches == wr.stats.failed_batches == (0 if quarantine else 3)
    assert_same(snapshot(col, ids), snapshot(wr.store, ids), 2e-3)
    wo, _ = run(MemoryStore(), "native", quarantine=quarantine, fault_poison=poison)  # object path
    assert sorted(m.body for m in wo.rabbit.drain("analyze_failed")) == failed_r
    assert_same(snapshot(wo.store, ids), snapshot(wr.store, ids), 2e-3)
