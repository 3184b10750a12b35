"""Batched engine (C++ host mirror) == per-object reference-semantics rater."""
import numpy as np
import pytest
import torch

from analyzer_amd.config import RaterConfig
from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream

from engine_parity import _stateful_slots, assert_engine_matches, object_run

SPECS = {
    "3v3": (RosterSpec(num_players=64, seed=5), StreamSpec(team_size=3, seed=11), 3),
    "5v5_edge": (RosterSpec(num_players=40, seed=6, p_tier_null=0.05, p_tier_bad=0.05,
                            p_rated=0.3),
                 StreamSpec(team_size=5, seed=12, p_tie=0.1, p_afk=0.05, p_uneven=0.2,
                            p_bad_rosters=0.03, p_unsupported=0.05,
                            modes={"5v5_casual": 0.5, "5v5_ranked": 0.5}), 5),
    "1v1_empty": (RosterSpec(num_players=12, seed=7),
                  StreamSpec(team_size=1, seed=13, p_uneven=0.2, p_tie=0.2), 1),
    "uneven_K4": (RosterSpec(num_players=30, seed=8, p_rated=0.0),
                  StreamSpec(team_size=4, seed=14, p_uneven=0.5), 4),
}


@pytest.mark.parametrize("name", sorted(SPECS))
def test_host_engine_matches_object_rater(name):
    rspec, sspec, K = SPECS[name]
    roster = make_roster(rspec)
    rec = make_stream(sspec, 400, rspec.num_players, K=K)
    ref = object_run(roster, rec, K)
    work = roster.clone()
    res = R.BatchRater(RaterConfig(), host_fp64=True).rate(work, rec, K)
    assert_engine_matches(res, work, ref, rtol=2e-6, atol_mu=2e-3, atol_delta=2e-3)


def test_host_engine_fp32_close_to_fp64():
    rspec, sspec, K = SPECS["3v3"]
    roster = make_roster(rspec)
    rec = make_stream(sspec, 400, rspec.num_players, K=K)
    a, b = roster.clone(), roster.clone()
    r64 = R.BatchRater(host_fp64=True).rate(a, rec, K)
    r32 = R.BatchRater(host_fp64=False).rate(b, rec, K)
    np.testing.assert_array_equal(r64.status.numpy(), r32.status.numpy())
    np.testing.assert_allclose(r32.s_mu.numpy(), r64.s_mu.numpy(), rtol=1e-4, equal_nan=True)


def test_stream_generator_properties():
    rec = make_stream(StreamSpec(team_size=3, seed=3, p_afk=0.0, p_tie=0.0), 5000, 1000)
    assert rec.shape == (5000, 8)
    ids = rec[:, :6]
    assert int(ids.min()) >= 0 and int(ids.max()) < 1000
    meta0 = rec[:, 6]
    assert bool(((meta0 >> 8) & 0xFF).eq(3).all())
    modes = (meta0 & 0xFF)
    counts = torch.bincount(modes, minlength=6)
    assert counts[1] > counts[2] > 0  # ranked 40% > blitz 15%
    w = rec[:, 7] & 3
    assert bool(((w == 1) | (w == 2)).all())
    # same seed -> same stream, different base -> different stream
    assert torch.equal(rec, make_stream(StreamSpec(team_size=3, seed=3, p_afk=0.0, p_tie=0.0), 5000, 1000))
    other = make_stream(StreamSpec(team_size=3, seed=3, p_afk=0.0, p_tie=0.0), 5000, 1000, base=5000)
    assert not torch.equal(rec, other)


def test_schedule_links_host():
    from analyzer_amd.ops.rate import BatchRater, Schedule

    rec = make_stream(StreamSpec(team_size=3, seed=9, p_afk=0.1), 300, 20)
    link, deps = BatchRater().schedule(rec, 3, 20)
    link = link.numpy().reshape(-1).astype(np.int64) & 0xFFFFFFFF
    deps = deps.numpy()
    occ = {}  # player -> [(match, slot)] in stream order
    expect_deps = np.zeros(rec.shape[0], dtype=np.int64)
    for m in range(rec.shape[0]):
        if int(rec[m, 7]) & 4:  # AFK: no state, not scheduled
            assert deps[m] == 0
            continue
        seen_here = set()
        for j in range(6):
            pid = int(rec[m, j])
            if pid not in seen_here:
                seen_here.add(pid)
                expect_deps[m] += pid in occ
            occ.setdefault(pid, []).append((m, m * 6 + j))
    assert (deps == expect_deps).all()
    for pid, lst in occ.items():
        for i, (m, slot) in enumerate(lst):
            w = int(link[slot])
            nxt = lst[i + 1][0] if i + 1 < len(lst) else Schedule.NO_MATCH
            assert w & Schedule.MATCH_MASK == nxt
            assert bool(w & Schedule.HAS_PRED) == (i > 0)


def test_status_counts_and_any_afk():
    rspec, sspec, K = SPECS["5v5_edge"]
    roster = make_roster(rspec)
    rec = make_stream(sspec, 300, rspec.num_players, K=K)
    res = R.BatchRater().rate(roster, rec, K)
    counts = res.status_counts()
    assert counts.get("rated", 0) > 0 and counts.get("afk", 0) > 0
    assert bool(res.any_afk[res.status == R.AFK].all())
    assert torch.isnan(res.quality[res.status == R.UNSUPPORTED_MODE]).all()
    assert (res.quality[res.status == R.AFK] == 0).all()


def test_noop_padding_records_touch_nothing():
    """The graph rater pads short batches with 'unsupported mode' records
    (ops/graph.py): they rate as UNSUPPORTED_MODE and leave the roster alone."""
    from analyzer_amd.ops.graph import noop_records

    K, P = 3, 50
    roster = make_roster(RosterSpec(num_players=P, seed=3))
    before = roster.state.clone()
    rec = torch.cat([noop_records(7, K, "cpu"),
                     make_stream(StreamSpec(team_size=K, seed=4), 5, P, K=K),
                     noop_records(3, K, "cpu")])
    ref = make_roster(RosterSpec(num_players=P, seed=3))
    res = R.BatchRater().rate(roster, rec, K)
    exp = R.BatchRater().rate(ref, rec[7:12], K)
    assert (res.status[:7] == R.UNSUPPORTED_MODE).all() and (res.status[12:] == R.UNSUPPORTED_MODE).all()
    assert torch.equal(res.status[7:12], exp.status)
    assert torch.equal(roster.state.nan_to_num(-7), ref.state.nan_to_num(-7))
    assert not torch.equal(roster.state.nan_to_num(-7), before.nan_to_num(-7))


def test_grid_blocks_scale_with_the_window():
    br = R.BatchRater(blocks=512)
    assert br.chunk_len(500) == 8 and br.grid_blocks(500) == 16   # 63 chunks of 8 -> 63 waves
    assert br.chunk_len(500, telemetry=True) == 64
    assert br.chunk_len(20_000) == 16 and br.chunk_len(10_000_000) == 64
    assert br.grid_blocks(1) == 1
    assert br.chunk_len(25_600) == 16 and br.grid_blocks(25_600) == 400  # 1600 chunks of 16
    assert br.chunk_len(64 * 2048 * 2) == 64 and br.grid_blocks(64 * 2048 * 2) == 512
    assert br.grid_blocks(10_000_000) == 512
    assert br.grid_blocks(500, telemetry=True) == 512
    # 5v5 windows take 32-match chunks (ANA_RATE_CHUNK caps any team size)
    assert br.chunk_len(10_000_000, K=5) == 32 and br.chunk_len(10_000_000, K=4) == 64
    assert br.grid_blocks(64 * 2048, K=5) == 512 and br.grid_blocks(32 * 2048, K=5) == 512
    assert br.chunk_len(500, K=5) == 8 and br.chunk_len(500, telemetry=True, K=5) == 64


@pytest.mark.parametrize("skew", [1, 2, 3])
def test_skewed_activity_draw(skew):
    """``StreamSpec.skew``: player = floor(u^skew * P), so P(player < x) = (x/P)^(1/skew)."""
    from analyzer_amd.ops.synth import StreamSpec, make_stream

    P, M = 100_000, 40_000
    rec = make_stream(StreamSpec(team_size=3, seed=5, p_afk=0.0, skew=skew), M, P)
    ids = rec[:, :6].reshape(-1).double()
    for x in (100, 10_000):
        frac = float((ids < x).double().mean())
        assert abs(frac - (x / P) ** (1.0 / skew)) < 0.01, (x, frac)


def test_prepass_placement_knob():
    """ANA_PREPASS_SERIAL: 1/0 force the placement; unset or auto -> serial for 4v4 and 5v5
    at two waves per SIMD; the executor grid per launch (BatchRater.launch_blocks)."""
    from analyzer_amd.config import EngineConfig
    from analyzer_amd.runtime.engine import WindowPipeline

    auto = EngineConfig.from_env({})
    assert auto.prepass_serial is None and EngineConfig.from_env({"ANA_PREPASS_SERIAL": "auto"}).prepass_serial is None
    assert WindowPipeline.serial_prepass(4, auto) and WindowPipeline.serial_prepass(5, auto)
    assert not WindowPipeline.serial_prepass(5, auto, dp=True)  # between DP merges: the probe decides
    # 1v1-3v3 launches leave a sort workgroup room at either grid (csrc/dataflow.hip ANA_EXEC_WPE)
    assert not WindowPipeline.serial_prepass(3, auto) and WindowPipeline.tail_point(3, auto) == 0.1
    # ... which assumes the 128-VGPR build: fused telemetry / the timing build launch uncapped
    assert WindowPipeline.tail_point(3, auto, capped=False) == 0.7
    on, off = (EngineConfig.from_env({"ANA_PREPASS_SERIAL": v}) for v in ("1", "0"))
    assert WindowPipeline.serial_prepass(5, on) and not WindowPipeline.serial_prepass(3, off)
    assert auto.prepass_at == 0.7 and EngineConfig.from_env({"ANA_PREPASS_AT": "0"}).prepass_at == 0.0
    # DP merges: short windows between merges overlap the next prepass with the tail, from 0.9 (3v3)
    assert not WindowPipeline.serial_prepass(3, auto, dp=True) and WindowPipeline.serial_prepass(3, on, dp=True)
    assert WindowPipeline.tail_point(3, auto, dp=True) == 0.9 and WindowPipeline.tail_point(5, auto, dp=True) == 0.9
    assert WindowPipeline.tail_point(3, EngineConfig.from_env({"ANA_PREPASS_AT": "0.5"}), dp=True) == 0.5
    assert WindowPipeline.tail_point(4, auto) == 0.7
    # one wave per SIMD (256 workgroups: <= 3v3 over a cached roster): the tail overlap from 0.55
    assert not WindowPipeline.serial_prepass(3, auto, grid=256) and WindowPipeline.serial_prepass(3, on, grid=256)
    assert WindowPipeline.tail_point(3, auto, grid=256) == 0.55 and WindowPipeline.tail_point(3, auto, dp=True, grid=256) == 0.9
    from analyzer_amd.ops.rate import BatchRater

    br = BatchRater()
    assert br.launch_blocks(3, 128 << 20) == 256 and br.launch_blocks(3, 1280 << 20) == 512
    assert br.launch_blocks(5, 128 << 20) == 256 and br.launch_blocks(4, 1280 << 20) == 512
    assert BatchRater(blocks=384).launch_blocks(3, 0) == 384
    # 4v4 / 5v5 over a cached roster: one wave per SIMD, the prepass overlapped (5v5 from 0.5)
    assert not WindowPipeline.serial_prepass(5, auto, grid=256) and WindowPipeline.tail_point(5, auto, grid=256) == 0.5
    assert not WindowPipeline.serial_prepass(4, auto, grid=256) and WindowPipeline.tail_point(4, auto, grid=256) == 0.55
    assert not auto.roster_warm and EngineConfig.from_env({"ANA_ROSTER_WARM": "1"}).roster_warm


def test_warm_rows_host_is_a_no_op():
    """warm_rows on a host roster checks its operands and changes nothing."""
    from analyzer_amd.ops.native import native

    roster = make_roster(RosterSpec(num_players=64, seed=5))
    before = roster.state.clone()
    native().warm_rows(roster.state, torch.zeros(256, dtype=torch.int32))
    assert torch.equal(roster.state.nan_to_num(-7), before.nan_to_num(-7))
    with pytest.raises(RuntimeError):
        native().warm_rows(roster.state, torch.zeros(8, dtype=torch.int32))

