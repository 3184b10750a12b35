"""K8 telemetry aggregation: generator, host mirror vs numpy oracle, fused launch
(CPU here; the device kernels are covered in test_engine_gpu.py)."""
import numpy as np
import torch

from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
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
