"""K8 telemetry aggregation: generator, host mirror vs numpy oracle, fused launch
(CPU here; the device kernels are covered in test_engine_gpu.py)."""
import numpy as np
import pytest
import torch

from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from analyzer_amd.runtime.objects import STAT_COLUMNS
from analyzer_amd.ops.telemetry import (STAT_NAMES, TelemetrySpec, aggregate, aggregate_reference,
                                        allocate_stats, make_telemetry)


def _stream(M=300, K=3, P=50, seed=3, **kw):
    return make_stream(StreamSpec(team_size=K, seed=seed, **kw), M, P, K=K)


def test_generator_layout_and_determinism():
    K = 3
    rec = _stream(p_uneven=0.3)
    tel = make_telemetry(TelemetrySpec(seed=5, min_events=10, max_events=40), rec, K)
    counts = (tel.evoff[1:] - tel.evoff[:-1]).numpy()
    assert counts.min() >= 10 and counts.max() <= 40 and tel.num_events == counts.sum()
    ev = tel.events.numpy()
    m = np.repeat(np.arange(rec.shape[0]), counts)
    assert ((ev[:, 0] >> 16) & 0xFFFF == m & 0xFFFF).all()  # 16-bit match tag
    slot = ev[:, 0] & 0xFF
    n0 = ((rec[:, 6] >> 8) & 0xFF).numpy()[m]
    n1 = ((rec[:, 6] >> 16) & 0xFF).numpy()[m]
    assert (((slot < n0)) | ((slot >= K) & (slot < K + n1))).all()  # real participants only
    again = make_telemetry(TelemetrySpec(seed=5, min_events=10, max_events=40), rec, K)
    assert torch.equal(tel.events, again.events)
    # the events of a match depend on its global index only
    tail = make_telemetry(TelemetrySpec(seed=5, min_events=10, max_events=40), rec[100:], K, base=100)
    o = int(tel.evoff[100])
    assert torch.equal(tail.events[:, 1], tel.events[o:, 1])                   # values
    assert torch.equal(tail.events[:, 0] & 0xFFFF, tel.events[o:, 0] & 0xFFFF)  # slot, type


def test_host_aggregation_matches_oracle():
    K = 5
    rec = _stream(M=200, K=K, P=80, seed=4)
    tel = make_telemetry(TelemetrySpec(seed=9), rec, K)
    got = aggregate(tel, K).numpy()
    ref = aggregate_reference(tel, K)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-2)
    assert got[..., STAT_NAMES.index("events")].sum() == tel.num_events


def test_fused_rate_gives_same_stats_and_ratings():
    K = 3
    roster = make_roster(RosterSpec(num_players=40, seed=2))
    rec = _stream(M=250, K=K, P=40, seed=8)
    tel = make_telemetry(TelemetrySpec(seed=1), rec, K)
    stats = allocate_stats(rec.shape[0], K, "cpu")
    a, b = roster.clone(), roster.clone()
    ra = R.BatchRater().rate(a, rec, K, telemetry=(tel.evoff, tel.events, stats))
    rb = R.BatchRater().rate(b, rec, K)
    assert torch.equal(a.state.nan_to_num(-7), b.state.nan_to_num(-7))
    assert torch.equal(ra.s_mu.nan_to_num(-7), rb.s_mu.nan_to_num(-7))
    np.testing.assert_allclose(stats.numpy(), aggregate_reference(tel, K), rtol=1e-5, atol=1e-2)


def test_malformed_events_are_dropped_and_counted():
    K = 1
    rec = _stream(M=20, K=K, P=10, seed=6)
    tel = make_telemetry(TelemetrySpec(seed=2, min_events=3, max_events=3), rec, K)
    ev = tel.events.clone()
    ev[0, 0] = (ev[0, 0] & ~0xFF) | 7                     # slot 7 >= 2K
    ev[5, 0] = (ev[5, 0] & 0xFFFF) | (19 << 16)            # names a match in another tile
    from analyzer_amd.ops.native import native
    stats = allocate_stats(20, K, "cpu")
    bad = native().telemetry(tel.evoff, ev, K, stats, torch.zeros(1, dtype=torch.int32))
    assert bad == 2
    assert stats[..., 7].sum() == tel.num_events - 2


def test_strict_attribution_same_tile_other_match():
    """An event counts only for the match whose CSR range holds it: naming another
    match of the same 16-match tile is malformed too (host mirror = device rule)."""
    K = 1
    rec = _stream(M=20, K=K, P=10, seed=7)
    tel = make_telemetry(TelemetrySpec(seed=3, min_events=2, max_events=2), rec, K)
    ev = tel.events.clone()
    ev[4, 0] = (ev[4, 0] & 0xFFFF) | (3 << 16)  # event of match 2 names match 3 (same tile)
    from analyzer_amd.ops.native import native
    stats = allocate_stats(20, K, "cpu")
    bad = native().telemetry(tel.evoff, ev, K, stats, torch.zeros(1, dtype=torch.int32))
    assert bad == 1
    assert stats[2, :, 7].sum() == 1 and stats[3, :, 7].sum() == 2


# ------------------------------------------------------------------ real event files
def _events_for(store, ids, seed=3):
    """Random downloaded-telemetry events for stored matches: (roster, position,
    type, value) per event, some matches without any, some events malformed
    (a third roster's participant, a position beyond the team)."""
    rng = np.random.default_rng(seed)
    s = store.session()
    out, want = [], {}
    for m in s.load_matches(ids):
        if rng.random() < 0.15:
            continue  # no telemetry downloaded for this match
        evs = []
        for _ in range(int(rng.integers(0, 40))):
            r = int(rng.integers(0, 2))
            parts = m.rosters[r].participants if r < len(m.rosters) else []
            pos = int(rng.integers(0, len(parts) + (1 if rng.random() < 0.05 else 0))) if parts else 0
            typ = int(rng.integers(0, 8))
            val = float(np.float32(rng.uniform(0, 500)))
            evs.append((r, pos, typ, val))
            if pos < len(parts):
                st = want.setdefault(parts[pos].api_id, [0.0] * 8)
                if typ <= 2:
                    st[typ] += 1.0
                elif typ <= 6:
                    st[typ] += val
                st[7] += 1.0
        out.append((m.api_id, evs))
    s.close()
    return out, want


@pytest.mark.parametrize("uri", ["columnar://", "sqlite:///{tmp}/t.db", "sqlalchemy+sqlite:///{tmp}/sa.db"])
def test_worker_aggregates_events_from_a_telemetry_file(tmp_path, uri):
    """DOTELEMETRY with TELEMETRY_SOURCE: a real store (no SYNTHETIC_TELEMETRY)
    gets participant_stats aggregated from the events written to the file --
    round trip file -> worker -> store, per participant; the reflected
    SQLAlchemy store through its columnar batch path (runtime/sqla.py)."""
    _telemetry_file_roundtrip(tmp_path, uri)


@pytest.mark.gpu
def test_worker_telemetry_file_on_device(gpu_device, tmp_path):
    """The same round trip with the fused rating + aggregation launch on the GPU
    (pinned gather, asynchronous upload)."""
    _telemetry_file_roundtrip(tmp_path, "columnar://", device_check=True)


def _telemetry_file_roundtrip(tmp_path, uri, device_check=False):
    from analyzer_amd.config import RaterConfig, WorkerConfig
    from analyzer_amd.ops.telemetry import TelemetrySource, jsonl_to_telemetry
    from analyzer_amd.runtime import broker as B
    from analyzer_amd.runtime.source import populate, publish
    from analyzer_amd.runtime.store import open_store
    from analyzer_amd.runtime.worker import Worker
    import json

    uri = uri.format(tmp=tmp_path)
    store = open_store(uri)
    ms = populate(store, 60, 40, team_size=3, seed=2)
    ids = [m if isinstance(m, str) else m.api_id for m in ms]
    evs, want = _events_for(store, ids)
    with open(tmp_path / "ev.jsonl", "w") as f:
        for mid, e in evs:
            f.write(json.dumps({"match": mid, "events": [list(x) for x in e]}) + "\n")
    path = str(tmp_path / "ev.anatel")
    assert jsonl_to_telemetry(str(tmp_path / "ev.jsonl"), path) == sum(len(e) for _, e in evs)
    assert TelemetrySource(path).num_matches == len(evs)
    clock = B.ManualClock()
    cfg = WorkerConfig(batchsize=16, idle_timeout=1.0, engine="native", database_uri=uri, dotelemetry=True,
                       telemetry_source=path, resident=True)
    w = Worker(cfg, store=store, broker=B.MemoryBroker(clock), rater_cfg=RaterConfig(), clock=clock)
    w.connect()
    publish(w.channel, "analyze", ids)
    w.start_consuming()
    assert w.stats.acked == 60
    if device_check:
        assert w._batched().device.type == "cuda"
    s = store.session()
    n = 0
    for m in s.load_matches(ids):
        for p in m.participants:
            got = s.participant_stats(p.api_id)
            exp = want.get(p.api_id, [0.0] * 8)
            assert got is not None, p.api_id
            np.testing.assert_allclose([got[c] for c in STAT_COLUMNS], exp, rtol=1e-5, atol=1e-3)
            n += exp[7] > 0
    assert n > 100


def test_synthetic_guard_only_without_a_source(tmp_path):
    from analyzer_amd.config import WorkerConfig
    from analyzer_amd.ops.telemetry import write_telemetry
    from analyzer_amd.runtime import broker as B
    from analyzer_amd.runtime.worker import Worker

    uri = "sqlite:///" + str(tmp_path / "g.db")
    with pytest.raises(ValueError, match="SYNTHETIC"):
        Worker(WorkerConfig(engine="native", database_uri=uri, dotelemetry=True),
               broker=B.MemoryBroker()).connect()
    path = str(tmp_path / "e.anatel")
    write_telemetry(path, [("m0", [(0, 0, "kill", 0.0)])])
    Worker(WorkerConfig(engine="native", database_uri=uri, dotelemetry=True, telemetry_source=path),
           broker=B.MemoryBroker()).connect()


def test_fuse_threshold_policy(monkeypatch):
    """Inline (fused) aggregation up to ANA_TELE_FUSE_MAX matches per launch, the
    MFMA kernel after the rating above it (scripts/tele_batch.py crossover);
    aggregation tiles (ANA_TELE_ROLE >= 0) are always fused."""
    import torch
    from analyzer_amd.ops import rate as R

    t = (torch.zeros(3, dtype=torch.int64), torch.zeros(0, 2, dtype=torch.int32), torch.zeros(0))
    br = R.BatchRater()
    assert br.tele_fuse_max == 262_144
    assert br.fuses(t, 500) and br.fuses(t, 262_144) and not br.fuses(t, 10_000_000)
    assert not br.tiles(t, 500) and not br.fuses(None, 500)
    monkeypatch.setenv("ANA_TELE_FUSE_MAX", "1000")
    assert not R.BatchRater().fuses(t, 1001)
    monkeypatch.setenv("ANA_TELE_ROLE", "2")
    br = R.BatchRater()
    assert br.tiles(t, 10_000_000) and br.fuses(t, 10_000_000)
