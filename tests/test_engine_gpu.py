"""MI355X kernels vs the C++ host mirror / object rater (numerics tests, ``-m gpu``)."""
import os

import numpy as np
import pytest
import torch

from analyzer_amd.config import RaterConfig
from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream

from engine_parity import _stateful_slots, assert_engine_matches, object_run
from test_engine_host import SPECS

pytestmark = pytest.mark.gpu


def assert_close_to_fp64(rd, dev, rh, host):
    """Device (fp32 state, hardware rcp/sqrt) vs the fp64 host mirror: within ~2x
    the deviation the 10M-match verification measures (ops/verify.py; max |d mu|
    0.0029, |d delta| 0.0005, relative d sigma 2.5e-6)."""
    for k, atol in (("s_mu", 6e-3), ("m_mu", 6e-3), ("delta", 1e-3)):
        np.testing.assert_allclose(getattr(rd, k).cpu().numpy(), getattr(rh, k).numpy(), rtol=0,
                                   atol=atol, equal_nan=True, err_msg=k)
    for k in ("s_sig", "m_sig"):
        np.testing.assert_allclose(getattr(rd, k).cpu().numpy(), getattr(rh, k).numpy(), rtol=5e-6,
                                   atol=0, equal_nan=True, err_msg=k)
    np.testing.assert_allclose(rd.quality.cpu().numpy(), rh.quality.numpy(), rtol=0, atol=2e-6,
                               equal_nan=True)
    td, th = dev.tracks().cpu().numpy(), host.tracks().numpy()
    np.testing.assert_allclose(td[..., 0], th[..., 0], rtol=0, atol=6e-3, equal_nan=True)
    np.testing.assert_allclose(td[..., 1], th[..., 1], rtol=5e-6, atol=0, equal_nan=True)


def test_native_module_is_loaded(gpu_device):
    from analyzer_amd.ops.native import native

    mod = native()
    assert mod.__file__.startswith(__import__("os").path.dirname(__import__("analyzer_amd").__file__))


def test_generators_bit_identical(gpu_device):
    rs = RosterSpec(num_players=5000, seed=21, p_tier_null=0.1, p_tier_bad=0.1)
    a, b = make_roster(rs), make_roster(rs, device=gpu_device)
    assert torch.equal(a.state.view(torch.int32), b.state.cpu().view(torch.int32))
    assert torch.equal(a.attrs.view(torch.int32), b.attrs.cpu().view(torch.int32))
    for K, skew in ((1, 1), (3, 1), (5, 1), (3, 2), (3, 3)):
        ss = StreamSpec(team_size=K, seed=33, p_afk=0.1, p_tie=0.1, p_hot=0.3, p_uneven=0.1, skew=skew)
        ra = make_stream(ss, 20000, 5000, base=123)
        rb = make_stream(ss, 20000, 5000, base=123, device=gpu_device)
        assert torch.equal(ra, rb.cpu())


# 1 (P=20), 2 (P=300, 5000), 3 (P=70k) and 4 (P=17M) radix passes: every
# combination of the fused first / last passes of the schedule sort
# + micro-batches (<= 8192 slots): the one-workgroup LDS bitonic schedule
@pytest.mark.parametrize("P,M,K", [(20, 3000, 3), (5000, 100000, 3), (300, 20000, 5),
                                   (70_000, 400_000, 3), (17_000_000, 300_000, 3),
                                   (50, 400, 3), (5000, 819, 5), (1_000_000, 1365, 3), (20, 1, 1),
                                   (40, 700, 2)])
def test_schedule_matches_host(gpu_device, P, M, K):
    ss = StreamSpec(team_size=K, seed=P, p_afk=0.05, p_unsupported=0.05, p_uneven=0.05, p_hot=0.2)
    rec = make_stream(ss, M, P, K=K)
    br = R.BatchRater()
    link_h, deps_h = (t.clone() for t in br.schedule(rec, K, P))
    link_d, deps_d = br.schedule(rec.to(gpu_device), K, P)
    slots, first = _stateful_slots(rec.numpy(), K, P)
    link_d = link_d.cpu().numpy()
    np.testing.assert_array_equal(link_d[slots], link_h.numpy()[slots])
    # device counters start at 0; the executor's readiness count comes from the links
    assert int(deps_d.abs().sum()) == 0
    need = (first & ((link_d & R.Schedule.HAS_PRED) != 0)).sum(1)
    rated = slots.any(1)
    np.testing.assert_array_equal(need[rated], deps_h.numpy()[rated])


@pytest.mark.parametrize("P,M,K,skew,runs,rb", [(1_000_000, 400_000, 3, 3, "1", "8"),
                                                (1_000_000, 400_000, 3, 1, "0", "8"),
                                                (1_000_000, 400_000, 3, 1, "1", "8"),
                                                (5000, 300_000, 5, 2, "1", "8"),
                                                (5000, 300_000, 3, 2, "1", "10"),
                                                (300_000, 400_000, 3, 1, "1", "10")])
def test_schedule_run_table_matches_host(gpu_device, P, M, K, skew, runs, rb, monkeypatch):
    """The last sort pass with run ends in a [tile][digit] table (no digit offsets,
    sched_runs_fixup) and the round-2 path (ANA_SCHED_RUNS=0): the same links as the
    host, also on power-law streams where a hot player's runs span many tiles and a
    sparse player's nearest earlier run lies tiles back.  ANA_SORT_RB=10 (10-bit
    digits, read per schedule): a small roster's single pass (<= 1024 digits) and a
    two-pass one, both through the run table."""
    monkeypatch.setenv("ANA_SCHED_RUNS", runs)
    monkeypatch.setenv("ANA_SORT_RB", rb)
    rec = make_stream(StreamSpec(team_size=K, seed=P + skew, skew=skew, p_afk=0.05), M, P, K=K)
    br = R.BatchRater()
    link_h, deps_h = (t.clone() for t in br.schedule(rec, K, P))
    link_d, deps_d = br.schedule(rec.to(gpu_device), K, P)
    slots, first = _stateful_slots(rec.numpy(), K, P)
    link_d = link_d.cpu().numpy()
    np.testing.assert_array_equal(link_d[slots], link_h.numpy()[slots])
    assert int(deps_d.abs().sum()) == 0


@pytest.mark.parametrize("P,M,K", [(20, 3000, 3), (70_000, 400_000, 3), (17_000_000, 300_000, 5)])
def test_schedule_link_parts_match_host(gpu_device, P, M, K, monkeypatch):
    """The link pass split into slot-range parts (ANA_LINK_PARTS; automatic above
    256 MB of links) writes the same links and boundary pairs as one pass."""
    monkeypatch.setenv("ANA_LINK_PARTS", "3")
    rec = make_stream(StreamSpec(team_size=K, seed=P + 5, p_afk=0.05, p_hot=0.2, p_uneven=0.05), M, P, K=K)
    br = R.BatchRater()
    link_h, deps_h = (t.clone() for t in br.schedule(rec, K, P))
    link_d, deps_d = br.schedule(rec.to(gpu_device), K, P)
    slots, first = _stateful_slots(rec.numpy(), K, P)
    link_d = link_d.cpu().numpy()
    np.testing.assert_array_equal(link_d[slots], link_h.numpy()[slots])
    need = (first & ((link_d & R.Schedule.HAS_PRED) != 0)).sum(1)
    rated = slots.any(1)
    np.testing.assert_array_equal(need[rated], deps_h.numpy()[rated])


@pytest.mark.parametrize("name", sorted(SPECS))
def test_device_matches_object_rater(gpu_device, name):
    rspec, sspec, K = SPECS[name]
    roster = make_roster(rspec)
    # 20k matches over 12-64 players: every player carries a chain of hundreds to
    # thousands of updates.  fp32 state + the hardware rcp/sqrt paths stay within
    # ~2x the error the 10M-match bench verification measures (ops/verify.py:
    # max |d mu| 0.0029, |d delta| 0.0005, relative d sigma 2.5e-6, profiles/r2)
    rec = make_stream(sspec, 20000, rspec.num_players, K=K)
    ref = object_run(roster, rec, K)
    work = roster.to(gpu_device)
    res = R.BatchRater(RaterConfig()).rate(work, rec.to(gpu_device), K)
    assert_engine_matches(res, work, ref, rtol=3e-6, atol_mu=6e-3, atol_delta=1e-3)


@pytest.mark.parametrize("P,M,hot", [(16, 4000, 0.0), (2000, 300000, 0.3), (100000, 1000000, 0.0)])
def test_device_matches_host_under_contention(gpu_device, P, M, hot):
    """Heavy per-player chains (P=16: every match depends on the previous ones) and
    hot-set skew exercise the cross-workgroup hand-off; any stale read shows up here."""
    rs = RosterSpec(num_players=P, seed=P + 1)
    ss = StreamSpec(team_size=3, seed=M, p_hot=hot, hot_fraction=0.01)
    roster = make_roster(rs)
    rec = make_stream(ss, M, P)
    host = roster.clone()
    rh = R.BatchRater(host_fp64=True).rate(host, rec, 3)
    dev = roster.to(gpu_device)
    rd = R.BatchRater().rate(dev, rec.to(gpu_device), 3)
    np.testing.assert_array_equal(rd.status.cpu().numpy(), rh.status.numpy())
    assert_close_to_fp64(rd, dev, rh, host)


def test_device_repeat_launch_deterministic(gpu_device):
    rs = RosterSpec(num_players=1000, seed=4)
    rec = make_stream(StreamSpec(seed=5), 50000, 1000, device=gpu_device)
    outs = []
    for _ in range(2):
        ro = make_roster(rs, device=gpu_device)
        res = R.BatchRater().rate(ro, rec)
        outs.append((ro.state.cpu(), res.s_mu.cpu()))  # compare values, not tags
    assert torch.equal(outs[0][0][:, 0::2].contiguous().view(torch.int32),
                       outs[1][0][:, 0::2].contiguous().view(torch.int32))
    assert torch.equal(outs[0][1].view(torch.int32), outs[1][1].view(torch.int32))


@pytest.mark.parametrize("K", [4, 5])
def test_chunk_length_bit_identical(gpu_device, K):
    """4v4 / 5v5 windows at their default grid and chunk (5v5: 32-match tickets,
    ops/rate.py chunk_len) give the bits of 64- and 16-match tickets at 512 workgroups:
    the ticket size changes only when a match runs."""
    P, M = 100000, 400000
    rs = RosterSpec(num_players=P, seed=21)
    rec = make_stream(StreamSpec(team_size=K, seed=22), M, P, K=K, device=gpu_device)
    outs = []
    for blocks, cap in ((None, 0), (512, 64), (512, 16)):
        ro = make_roster(rs, device=gpu_device)
        rater = R.BatchRater(blocks=blocks)
        rater.chunk_cap = cap
        if blocks is None:
            assert rater.launch_blocks(K, ro.state.numel() * ro.state.element_size()) == 256
            assert rater.chunk_len(M, blocks=256, K=K) == (32 if K == 5 else 64)
        res = rater.rate(ro, rec, K)
        assert int(rater.error_flags(gpu_device).sum()) == 0
        outs.append((ro.state.cpu(), res.s_mu.cpu(), res.status.cpu(), res.m_sig.cpu()))
    a = outs[0]
    for b in outs[1:]:
        assert torch.equal(a[0][:, 0::2].contiguous().view(torch.int32), b[0][:, 0::2].contiguous().view(torch.int32))
        assert torch.equal(a[1].view(torch.int32), b[1].view(torch.int32))
        assert torch.equal(a[2], b[2])
        assert torch.equal(a[3].view(torch.int32), b[3].view(torch.int32))


@pytest.mark.parametrize("K", [2, 3])
def test_grid_and_register_builds_bit_identical(gpu_device, K):
    """The launch grid picks the build: at two waves per SIMD (> 256 workgroups) plain
    1v1-3v3 launches run the kernel compiled for 4 waves per SIMD (128 VGPRs,
    csrc/dataflow.hip WPE), at <= 256 the unconstrained one.  Grid and build change
    only when a match runs: every combination gives the bits of the 256-workgroup run."""
    P, M = 100000, 600000
    rs = RosterSpec(num_players=P, seed=11)
    rec = make_stream(StreamSpec(team_size=K, seed=12), M, P, K=K, device=gpu_device)
    outs = {}
    for blocks in (256, 512, 64):
        ro = make_roster(rs, device=gpu_device)
        rater = R.BatchRater(blocks=blocks)
        assert rater.launch_blocks(K, ro.state.numel() * ro.state.element_size()) == blocks
        res = rater.rate(ro, rec, K)
        assert int(rater.error_flags(gpu_device).sum()) == 0
        outs[blocks] = (ro.state.cpu(), res.s_mu.cpu(), res.status.cpu(), res.quality.cpu())
    a = outs[256]
    for blocks in (512, 64):
        b = outs[blocks]
        assert torch.equal(a[0][:, 0::2].contiguous().view(torch.int32),
                           b[0][:, 0::2].contiguous().view(torch.int32)), blocks
        assert torch.equal(a[1].view(torch.int32), b[1].view(torch.int32)), blocks
        assert torch.equal(a[2], b[2]), blocks
        assert torch.equal(a[3].view(torch.int32), b[3].view(torch.int32)), blocks


def _handoff_run(K, P, M, skew, device, expect_local):
    """Rate one stream with every (ANA_RATE_LOCAL, ANA_RATE_DIAG) setting; the results
    must be bit-identical, and the local hand-off must (or, where it is compiled out,
    must not) take hot chains."""
    rs = RosterSpec(num_players=P, seed=P + 3)
    rec = make_stream(StreamSpec(team_size=K, seed=M + 1, skew=skew), M, P, K=K, device=device)
    outs = []
    for local, diag in (("0", "0"), ("1", "0"), ("1", "1"), ("0", "1")):
        os.environ["ANA_RATE_LOCAL"] = local
        os.environ["ANA_RATE_DIAG"] = diag
        ro = make_roster(rs, device=device)
        rater = R.BatchRater()
        res = rater.rate(ro, rec, K)
        assert int(rater.error_flags(device).sum()) == 0
        nl, ng = rater.handoffs(device)
        if local == "0" or not expect_local:
            assert nl == 0, (local, nl)
        elif P <= 16 or skew > 1:
            assert nl > 0, (nl, ng)
        d = rater.diag(device)
        if diag == "1":
            assert d["worked_iterations"] > 0 and d["wait_us"] > 0.0 and d["after_us"] > 0.0, d
        outs.append((ro.state.cpu(), res.s_mu.cpu(), res.status.cpu(), res.quality.cpu()))
    for b in outs[1:]:
        a = outs[0]
        assert torch.equal(a[0][:, 0::2].contiguous().view(torch.int32),
                           b[0][:, 0::2].contiguous().view(torch.int32))
        assert torch.equal(a[1].view(torch.int32), b[1].view(torch.int32))
        assert torch.equal(a[2], b[2])
        assert torch.equal(a[3].view(torch.int32), b[3].view(torch.int32))


@pytest.mark.parametrize("K,P,M,skew", [(3, 16, 4000, 1), (3, 100000, 1000000, 1), (5, 2000, 200000, 1),
                                        (3, 100000, 300000, 3), (4, 50000, 300000, 3)])
def test_local_handoff_and_timing_build_bit_identical(gpu_device, monkeypatch, K, P, M, skew):
    """The timing build (ANA_RATE_DIAG) and the LDS local hand-off (ANA_RATE_LOCAL) change
    only WHEN a match runs, never its result.  The production library compiles the hand-off
    into the 1v1-4v4 executors only (csrc/dataflow.hip kLH): there hot chains take it, for
    5v5 setting it changes nothing and no hand-off goes local."""
    monkeypatch.setenv("ANA_RATE_LOCAL", "0")
    monkeypatch.setenv("ANA_RATE_DIAG", "0")
    _handoff_run(K, P, M, skew, gpu_device, expect_local=K <= 4)


def test_local_handoff_in_diagnostic_library(gpu_device):
    """The diagnostic library (_C_diag, ANA_DIAG_BUILD) keeps the local hand-off: hot
    chains (16 players, cubic skew) take it and every result is bit-identical (run in a
    child process: one library per process)."""
    import subprocess
    import sys

    from analyzer_amd.build_ext import target_path

    lib = str(target_path(diag=True))
    if not os.path.exists(lib):
        pytest.skip("diagnostic library not built (python -m analyzer_amd.build_ext --diag)")
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "import torch, test_engine_gpu as t\n"
            "for args in ((3, 16, 4000, 1), (3, 100000, 300000, 3)):\n"
            "    t._handoff_run(*args, torch.device('cuda:0'), True)\n"
            "print('ok')\n") % (os.path.dirname(os.path.abspath(__file__)),
                                 os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, ANA_NATIVE_LIB=lib)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]


@pytest.mark.parametrize("n,bits", [(1, 8), (4095, 20), (4097, 12), (1_000_003, 20), (300_000, 32)])
def test_radix_sort_pairs_stable(gpu_device, n, bits):
    from analyzer_amd.ops.native import native

    g = torch.Generator().manual_seed(n)
    hi = 1 << min(bits, 31)
    keys = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64)
    if bits == 32:
        keys = keys * 2 - hi  # negative int32 = high unsigned keys
    keys = keys.to(torch.int32)
    if n > 1000:
        keys[: n // 3] = keys[0]  # long equal runs exercise stability
    vals = torch.arange(n, dtype=torch.int32)
    ks, vs = native().sort_pairs(keys.to(gpu_device), vals.to(gpu_device), bits)
    ukeys = keys.to(torch.int64) & 0xFFFFFFFF
    order = torch.sort(ukeys, stable=True).indices
    assert torch.equal(ks.cpu(), keys[order])
    assert torch.equal(vs.cpu(), vals[order])


@pytest.mark.parametrize("scaled", [False, True])
@pytest.mark.parametrize("resweep", [False, True])
def test_sweep_kernels_match_host(gpu_device, scaled, resweep):
    """K9 device kernels (messages + decode, dual write; one lane per track over
    base rows) == C++ host mirror; ``resweep``: messages measured from a prior !=
    the start."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.models.tiers import vst_table
    from analyzer_amd.parallel.sweep import base_rows

    P = 5000
    start = make_roster(RosterSpec(num_players=P, seed=3, p_rated=0.5))
    prior = start.clone()
    if resweep:  # a prior that moved on from the start (touches NULL tracks too)
        R.BatchRater().rate(prior, make_stream(StreamSpec(team_size=3, seed=14), 8000, P), 3)
    after = prior.clone()
    rec = make_stream(StreamSpec(team_size=3, seed=4), 20000, P)
    R.BatchRater().rate(after, rec, 3)
    vst = torch.tensor(vst_table(), dtype=torch.float32)
    g = lambda t: t.to(gpu_device)
    sb, pb = base_rows(start.state).contiguous(), base_rows(prior.state).contiguous()
    bh = torch.empty((P, 16))
    native().sweep_delta(sb, pb, after.state, start.attrs, vst, 500.0, scaled, bh)
    bd = torch.empty((P, 16), device=gpu_device)
    native().sweep_delta(g(sb), g(pb), g(after.state), g(start.attrs), g(vst), 500.0, scaled, bd)
    # scaled messages are (pi/pi_b - pi0/pi_b, ...): a 1-ulp difference in a ratio near 1
    # is a large relative one in the message (they travel as fp16/bf16 anyway)
    np.testing.assert_allclose(bd.cpu().numpy(), bh.numpy(), rtol=1e-3 if scaled else 1e-6,
                               atol=1e-5 if scaled else 1e-9)
    sh, sh2 = start.state.clone(), torch.zeros_like(sb)
    native().sweep_apply(sb, bh * 2, start.attrs, sh, sh2, vst, 500.0, scaled)
    sd, sd2 = g(start.state).clone(), torch.zeros_like(g(sb))
    native().sweep_apply(g(sb), g(bh * 2), g(start.attrs), sd, sd2, g(vst), 500.0, scaled)
    # fp32 (tau / pi, 1 / sqrt(pi)): device fma contraction vs host rounding
    np.testing.assert_allclose(sd.cpu().numpy(), sh.numpy(), rtol=5e-5, atol=1e-6, equal_nan=True)
    assert torch.equal(base_rows(sd).nan_to_num(-7), sd2.nan_to_num(-7))
    assert torch.equal(base_rows(sh).nan_to_num(-7), sh2.nan_to_num(-7))


@pytest.mark.parametrize("comm", ["fp32", "bf16", "fp16"])
def test_record_correction_kernel_matches_host(gpu_device, comm):
    """K9 causal record correction (one thread per slot): device == host mirror on a
    rated window's records, NULL tracks, seeds, AFK / invalid matches and a prefix of
    real messages (another slice's evidence) in every wire format."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.parallel.sweep import COMM_DTYPES, SweepMerger

    P, M, K = 5000, 20000, 3
    rs = RosterSpec(num_players=P, seed=41, p_rated=0.4)
    start = make_roster(rs)
    other = start.clone()
    R.BatchRater().rate(other, make_stream(StreamSpec(team_size=K, seed=42), M, P, K=K), K)
    m = SweepMerger(P, "cpu", comm_dtype=comm, force=True)
    m.begin(start)
    m.messages(other)  # an earlier slice's messages against the start: the prefix
    g = lambda t: t.to(gpu_device)
    if comm == "fp32":  # raw: the prefix is the increment table
        dh = m.buf.clone()
        dd = g(dh)
    else:  # scaled: the delta table from the window start, host and device (standalone + fused decode)
        prefix = m.buf[:, :14].to(COMM_DTYPES[comm]).contiguous()
        dh = torch.empty(P, 16)
        native().prefix_delta(m.start, prefix, start.attrs, m.vst, 500.0, dh)
        dd = torch.empty((P, 16), device=gpu_device)
        native().prefix_delta(g(m.start), g(prefix), g(start.attrs), g(m.vst), 500.0, dd)
        fused = torch.empty((P, 16), device=gpu_device)
        msg = torch.zeros((P, 14), dtype=prefix.dtype, device=gpu_device)
        cnt = torch.zeros((P, 1), dtype=torch.int32, device=gpu_device)
        native().sweep_apply_packed(g(m.start), msg, cnt, g(start.attrs), g(start.state).clone(),
                                    g(m.start).clone(), g(m.vst), 500.0, None, g(prefix), fused)
        torch.cuda.synchronize()
        # (d_tau = pi_B (r_tau + mu_B r_pi) cancels: device fma vs host rounding)
        np.testing.assert_allclose(dd.cpu().numpy(), dh.numpy(), rtol=1e-4, atol=1e-9)
        assert torch.equal(fused.cpu(), dd.cpu())
    rec = make_stream(StreamSpec(team_size=K, seed=43, p_afk=0.05, p_uneven=0.05), M, P, K=K)
    ro = start.clone()
    out = R.BatchRater().rate(ro, rec, K)
    host = out.packed.clone()
    native().correct_records(rec, K, host, dh)
    dev = out.packed.to(gpu_device)
    native().correct_records(g(rec), K, dev, dd)
    torch.cuda.synchronize()
    changed = (host != out.packed) & ~torch.isnan(host)
    assert int(changed.sum()) > 10000  # the prefix moved most rated records
    np.testing.assert_allclose(dev.cpu().numpy(), host.numpy(), rtol=2e-6, atol=2e-3, equal_nan=True)


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_device_decode_counts_clamps_like_host(gpu_device, comm):
    """The merge decode kernels count every track held at the precision floor into the
    merger's sticky word, as the host mirror does, and write the same clamped rows."""
    from analyzer_amd.parallel.sweep import MergeClampError, SweepMerger

    P = 3000
    ro = make_roster(RosterSpec(num_players=P, seed=5, p_rated=1.0, p_mode_rated=1.0))
    outs = []
    for dev in ("cpu", gpu_device):
        m = SweepMerger(P, dev, comm_dtype=comm, force=True)
        r = ro.clone().to(dev)  # (Roster.to of the same device aliases the tensors)
        m.begin(r)
        idx = torch.arange(0, P, 7, device=dev)
        if comm == "fp32":
            m.buf.zero_()
            m.buf[idx, 0] = -2.0 / m.start[idx, 1] ** 2   # shared track: pi_b + d_pi < 0
            m.buf[idx, 4] = -1.0e-12                      # mode track 2: a loss it can take
            m.decode(r)
        else:
            m.msg.zero_()
            m.cnt.zero_()
            m.msg[idx, 0] = -1.25                         # 1 + r_pi < 0
            m.decode_packed(r)
        outs.append((m.clamp_hits(), r.state.cpu()))
        with pytest.raises(MergeClampError):
            m.check()
    assert outs[0][0] == outs[1][0] == len(range(0, P, 7))
    np.testing.assert_allclose(outs[1][1].numpy(), outs[0][1].numpy(), rtol=5e-5, atol=1e-6, equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_packed_sweep_kernels_match_fp32_path(gpu_device, dtype):
    """The compressed-operand merge kernels (messages straight into bf16/fp16 +
    int32, decode straight from them) == the fp32 kernels followed by torch's
    conversions, bit for bit."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.models.tiers import vst_table
    from analyzer_amd.parallel.sweep import base_rows

    P = 6000
    start = make_roster(RosterSpec(num_players=P, seed=5, p_rated=0.5), device=gpu_device)
    after = start.clone()
    R.BatchRater().rate(after, make_stream(StreamSpec(team_size=3, seed=6), 20000, P, device=gpu_device), 3)
    vst = torch.tensor(vst_table(), dtype=torch.float32, device=gpu_device)
    sb = base_rows(start.state).contiguous()
    buf = torch.empty((P, 16), device=gpu_device)
    native().sweep_delta(sb, sb, after.state, start.attrs, vst, 500.0, True, buf)
    msg = torch.empty((P, 14), dtype=dtype, device=gpu_device)
    cnt = torch.empty((P, 1), dtype=torch.int32, device=gpu_device)
    native().sweep_delta_packed(sb, sb, after.state, start.attrs, vst, 500.0, msg, cnt)
    assert torch.equal(msg.view(torch.int16), buf[:, :14].to(dtype).view(torch.int16))
    lohi = buf[:, 14:].to(torch.int32)  # the touch fields travel packed: lo | hi << 16
    assert torch.equal(cnt, lohi[:, :1] | (lohi[:, 1:] << 16))
    msg2, cnt2 = msg * 2, cnt * 2  # a "sum" of two ranks (nibble fields: no carry)
    joined = torch.cat([msg2.float(), (cnt2 & 0xffff).float(), (cnt2 >> 16).float()], dim=1)
    s_ref, s2_ref = start.state.clone(), torch.zeros_like(sb)
    native().sweep_apply(sb, joined, start.attrs, s_ref, s2_ref, vst, 500.0, True)
    s_p, s2_p = start.state.clone(), torch.zeros_like(sb)
    native().sweep_apply_packed(sb, msg2, cnt2, start.attrs, s_p, s2_p, vst, 500.0)
    assert torch.equal(s_p.nan_to_num(-7), s_ref.nan_to_num(-7))
    assert torch.equal(s2_p.nan_to_num(-7), s2_ref.nan_to_num(-7))
    assert torch.equal(s2_ref.nan_to_num(-7), base_rows(s_ref).nan_to_num(-7))


def test_telemetry_device_generator_and_aggregation(gpu_device):
    from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, aggregate_reference, make_telemetry

    K = 3
    rec = make_stream(StreamSpec(team_size=K, seed=21, p_uneven=0.2), 50000, 4000, K=K)
    spec = TelemetrySpec(seed=4, min_events=20, max_events=120)
    th = make_telemetry(spec, rec, K)
    td = make_telemetry(spec, rec.to(gpu_device), K)
    assert torch.equal(td.evoff.cpu(), th.evoff) and torch.equal(td.events.cpu(), th.events)
    sd = aggregate(td, K)
    np.testing.assert_allclose(sd.cpu().numpy(), aggregate_reference(th, K), rtol=2e-5, atol=0.05)


@pytest.mark.parametrize("impl", ["1", "0", "2"])
@pytest.mark.parametrize("K", [1, 2, 3, 4, 5])
def test_telemetry_impls_vs_oracle_edges(gpu_device, monkeypatch, K, impl):
    """K8 one-hot MFMA (impl 1), LDS-atomic (impl 0) tiles and one lane per stat row
    (impl 2, also bit-identical to the host mirror) vs an fp64 oracle:
    every team size (16-row blocks of 8/4/2/2/1 matches), empty matches, a
    partial last tile, malformed events (strict attribution) and non-finite
    values; the host mirror counts the same malformed events."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.ops.telemetry import Telemetry, TelemetrySpec, aggregate, make_telemetry

    monkeypatch.setenv("ANA_TELE_IMPL", impl)
    M = 4099
    rec = make_stream(StreamSpec(team_size=K, seed=40 + K, p_uneven=0.2), M, 3000, K=K)
    tel = make_telemetry(TelemetrySpec(seed=5, min_events=0, max_events=90), rec, K)
    ev = tel.events.clone()
    idx = torch.randperm(ev.shape[0], generator=torch.Generator().manual_seed(K))[:60]
    ev[idx[:20], 0] = (ev[idx[:20], 0] & ~0xFF) | (2 * K)            # slot out of range
    ev[idx[20:40], 0] = ev[idx[20:40], 0] + (1 << 16)                # tag names the next match
    ev[idx[40:50], 0] = (ev[idx[40:50], 0] & ~0xFF00) | (3 << 8)     # damage events ...
    ev[:, 1].view(torch.float32)[idx[40:50]] = float("inf")          # ... of infinite value
    evn = ev.numpy()
    seg = np.repeat(np.arange(M), np.diff(tel.evoff.numpy()))
    m = seg
    tag = (evn[:, 0] >> 16) & 0xFFFF
    slot, typ = evn[:, 0] & 0xFF, (evn[:, 0] >> 8) & 0xFF
    ok = (tag == seg & 0xFFFF) & (slot < 2 * K)
    val = evn[:, 1].view(np.float32).astype(np.float64)
    add, feat = np.where(typ <= 2, 1.0, val), np.where(typ <= 6, typ, -1)
    ref = np.zeros((M, 2 * K, 8))
    sel = ok & (feat >= 0)
    np.add.at(ref, (m[sel], slot[sel], feat[sel]), add[sel])
    np.add.at(ref, (m[ok], slot[ok], np.full(int(ok.sum()), 7)), 1.0)
    host = torch.zeros(M, 2 * K, 8)
    assert native().telemetry(tel.evoff, ev, K, host, torch.zeros(1, dtype=torch.int32)) == int((~ok).sum())
    bad = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    stats = torch.full((M, 2 * K, 8), -1.0, device=gpu_device)  # every entry must be written
    aggregate(Telemetry(tel.evoff.to(gpu_device), ev.to(gpu_device)), K, stats, bad)
    torch.cuda.synchronize()
    assert int(bad.item()) == int((~ok).sum())
    np.testing.assert_allclose(stats.cpu().numpy(), ref, rtol=2e-6, atol=1e-3)
    np.testing.assert_allclose(host.numpy(), ref, rtol=2e-6, atol=1e-3)
    if impl == "2":  # row sums in event order, as the host mirror: the same bits
        assert torch.equal(stats.cpu(), host)


def test_graph_rater_matches_eager(gpu_device):
    """Micro-batches replayed as one HIP graph (ops/graph.py) rate exactly like
    eager launches: every batch size up to the capacity, and across the epoch
    wrap (tag reset) of the device-side launch epoch."""
    from analyzer_amd.ops.graph import GraphRater

    K, P = 3, 20000
    roster = make_roster(RosterSpec(num_players=P, seed=11), device=gpu_device)
    ref = roster.clone()
    stream = make_stream(StreamSpec(team_size=K, seed=12, p_afk=0.05, p_tie=0.05), 6000, P, K=K,
                         device=gpu_device)
    gr = GraphRater(roster, K, capacity=512)
    br = R.BatchRater()
    off = 0
    for i, m in enumerate([500, 100, 512, 37, 400, 1, 512, 300]):
        if i == 5:
            gr.clock.bumps = gr.MAX_EPOCH - 2  # the next replays pass the wrap: tags reset
        batch = stream[off:off + m]
        off += m
        got = gr.rate(batch)
        gr.check()
        exp = br.rate(ref, batch, K)
        assert torch.equal(got.status, exp.status)
        for f in ("quality", "s_mu", "s_sig", "delta", "m_mu", "m_sig"):
            assert torch.equal(getattr(got, f).nan_to_num(-7), getattr(exp, f).nan_to_num(-7)), f
        assert torch.equal(roster.state[:, 0::2].nan_to_num(-7), ref.state[:, 0::2].nan_to_num(-7))


def test_telemetry_diagnostic_variants_need_the_diag_library(gpu_device, monkeypatch):
    """ANA_TELE_DEBUG / non-default ANA_TELE_SPAN name kernel variants that only the
    diagnostic build (build_ext --diag) contains: the production library refuses them
    instead of timing its default kernel under their name."""
    from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, make_telemetry

    if os.environ.get("ANA_NATIVE_LIB"):
        pytest.skip("another library is loaded")
    rec = make_stream(StreamSpec(team_size=3, seed=3), 200, 100, K=3, device=gpu_device)
    tel = make_telemetry(TelemetrySpec(seed=1, min_events=5, max_events=9), rec, 3)
    ref = aggregate(tel, 3)
    for var, val in (("ANA_TELE_DEBUG", "7"), ("ANA_TELE_SPAN", "32")):
        monkeypatch.setenv(var, val)
        with pytest.raises(RuntimeError, match="diagnostic library"):
            aggregate(tel, 3)
        monkeypatch.delenv(var)
    assert torch.equal(aggregate(tel, 3), ref)


@pytest.mark.parametrize("role", [-1, 0, 2, 4, 8])
def test_fused_rate_telemetry_on_device(gpu_device, monkeypatch, role):
    """Fused aggregation: inline in the rating groups (role -1), idle-wave tiles
    (role 0) and dedicated aggregation waves (ANA_TELE_ROLE): same stats as the
    oracle, same ratings as without."""
    from analyzer_amd.ops.telemetry import (TelemetrySpec, aggregate_reference, allocate_stats,
                                            make_telemetry)

    monkeypatch.setenv("ANA_TELE_ROLE", str(role))
    monkeypatch.setenv("ANA_TELE_FUSE_MAX", str(1 << 30))  # inline even past the default threshold

    K, P, M = 3, 20000, 400000
    roster = make_roster(RosterSpec(num_players=P, seed=5), device=gpu_device)
    rec = make_stream(StreamSpec(team_size=K, seed=6), M, P, K=K, device=gpu_device)
    tel = make_telemetry(TelemetrySpec(seed=8, min_events=10, max_events=60), rec, K)
    stats = allocate_stats(M, K, gpu_device)
    a, b = roster.clone(), roster.clone()
    br = R.BatchRater()
    ra = br.rate(a, rec, K, telemetry=(tel.evoff, tel.events, stats))
    assert br.telemetry_errors(gpu_device) == 0
    rb = R.BatchRater().rate(b, rec, K)
    assert torch.equal(a.state.nan_to_num(-7), b.state.nan_to_num(-7))
    assert torch.equal(ra.s_mu.nan_to_num(-7), rb.s_mu.nan_to_num(-7))
    ref = aggregate_reference(type(tel)(tel.evoff.cpu(), tel.events.cpu()), K)
    np.testing.assert_allclose(stats.cpu().numpy(), ref, rtol=2e-5, atol=0.05)


@pytest.mark.parametrize("fuse_max", [1 << 30, 0])
def test_inline_telemetry_edge_cases_on_device(gpu_device, monkeypatch, fuse_max):
    """Inline aggregation (ANA_TELE_ROLE=-1) on the paths the common case skips:
    stateless matches (AFK, invalid rosters, unsupported) aggregated by tele-only
    groups, matches with more events than a group loads with its granules (the
    remainder loop), 5v5 groups, and malformed events counted, not folded.
    ``fuse_max`` 0: the same launch past ANA_TELE_FUSE_MAX, where BatchRater.rate
    runs the MFMA kernel after the rating -- same stats, ratings and error count."""
    from analyzer_amd.ops.telemetry import (TelemetrySpec, aggregate_reference, allocate_stats,
                                            make_telemetry)

    monkeypatch.setenv("ANA_TELE_ROLE", "-1")
    monkeypatch.setenv("ANA_TELE_FUSE_MAX", str(fuse_max))
    for K, lo, hi in ((3, 0, 150), (5, 30, 90)):
        P, M = 5000, 60000
        roster = make_roster(RosterSpec(num_players=P, seed=15), device=gpu_device)
        spec = StreamSpec(team_size=K, seed=16, p_afk=0.1, p_bad_rosters=0.05, p_unsupported=0.05,
                          p_tie=0.05)
        rec = make_stream(spec, M, P, K=K, device=gpu_device)
        tel = make_telemetry(TelemetrySpec(seed=18, min_events=lo, max_events=hi), rec, K)
        ev = tel.events.clone()
        ev[::97, 0] ^= 1 << 16  # wrong match tag: malformed
        stats = allocate_stats(M, K, gpu_device)
        a, b = roster.clone(), roster.clone()
        br = R.BatchRater()
        ra = br.rate(a, rec, K, telemetry=(tel.evoff, ev, stats))
        nbad = br.telemetry_errors(gpu_device)
        rb = R.BatchRater().rate(b, rec, K)
        assert torch.equal(a.state.nan_to_num(-7), b.state.nan_to_num(-7))
        assert torch.equal(ra.status, rb.status)
        for f in ("quality", "s_mu", "s_sig", "delta", "m_mu", "m_sig"):
            assert torch.equal(getattr(ra, f).nan_to_num(-7), getattr(rb, f).nan_to_num(-7)), f
        ref = aggregate_reference(type(tel)(tel.evoff.cpu(), ev.cpu()), K)
        np.testing.assert_allclose(stats.cpu().numpy(), ref, rtol=2e-5, atol=0.05)
        assert nbad == (ev.shape[0] + 96) // 97


def test_file_ingest_pipeline_on_device(gpu_device, tmp_path):
    """P3 on the GPU: native reader thread -> pinned ring -> H2D copy stream ->
    prepass/rate -> D2H copy stream; equals rating the stream in one launch."""
    from analyzer_amd.runtime.ingest import rate_file, write_records

    K, P, M = 3, 50000, 600000
    rec = make_stream(StreamSpec(team_size=K, seed=31), M, P, K=K)
    path = str(tmp_path / "s.rec")
    write_records(path, rec, K)
    roster = make_roster(RosterSpec(num_players=P, seed=32), device=gpu_device)
    direct = roster.clone()
    ref = R.BatchRater().rate(direct, rec.to(gpu_device), K)
    got = {}
    n = rate_file(path, roster, 100000, on_result=lambda b, h: got.__setitem__(b, h))
    assert n == 6
    s_mu = torch.cat([got[b]["s_mu"] for b in sorted(got)])
    torch.testing.assert_close(s_mu, ref.s_mu.cpu(), rtol=0, atol=0, equal_nan=True)
    torch.testing.assert_close(roster.tracks(), direct.tracks(), rtol=0, atol=0, equal_nan=True)


def test_roster_warm_pipeline_is_bit_identical(gpu_device, monkeypatch):
    """ANA_ROSTER_WARM: the warm-up read in front of each launch leaves the roster as it
    was and the windows rate bit-identically to a pipeline without it."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.runtime.engine import WindowPipeline

    K, P, M = 3, 20000, 120000
    roster = make_roster(RosterSpec(num_players=P, seed=41), device=gpu_device)
    before = roster.state.clone()
    sink = torch.zeros(256, dtype=torch.int32, device=gpu_device)
    native().warm_rows(roster.state, sink)
    torch.cuda.synchronize()
    assert torch.equal(roster.state.view(torch.int32), before.view(torch.int32))  # NaN = NULL: compare bits
    wins = [make_stream(StreamSpec(team_size=K, seed=42 + w), M, P, K=K, base=w * M).to(gpu_device)
            for w in range(3)]
    outs = {}
    for warm in ("0", "1"):
        monkeypatch.setenv("ANA_ROSTER_WARM", warm)
        r = roster.clone()
        pipe = WindowPipeline(R.BatchRater(), r, K)
        assert pipe.ecfg.roster_warm == (warm == "1")
        s_mu = []
        n = pipe.run(wins, on_result=lambda i, res: s_mu.append(res.s_mu.clone()))
        assert n == 3
        torch.cuda.synchronize()
        outs[warm] = (r.state.clone(), torch.cat(s_mu))
    assert torch.equal(outs["0"][0].nan_to_num(-7), outs["1"][0].nan_to_num(-7))
    assert torch.equal(outs["0"][1].nan_to_num(-7), outs["1"][1].nan_to_num(-7))


@pytest.mark.parametrize("case", ["empty", "one", "one_player", "all_afk", "all_unsupported",
                                  "all_bad_tier", "k5_uneven_ties"])
def test_edge_windows_device_vs_host(gpu_device, case):
    """Degenerate windows: the device executor terminates and matches the host mirror."""
    K, P, M = 3, 50, 400
    rspec = RosterSpec(num_players=P, seed=3)
    sspec = StreamSpec(team_size=K, seed=4)
    if case == "empty":
        M = 0
    elif case == "one":
        M = 1
    elif case == "one_player":
        P, rspec = 1, RosterSpec(num_players=1, seed=3)
    elif case == "all_afk":
        sspec = StreamSpec(team_size=K, seed=4, p_afk=1.0)
    elif case == "all_unsupported":
        sspec = StreamSpec(team_size=K, seed=4, p_unsupported=1.0)
    elif case == "all_bad_tier":
        rspec = RosterSpec(num_players=P, seed=3, p_rated=0.0, p_rp_ranked=0.0, p_rp_blitz=0.0,
                           p_tier_bad=1.0)
    elif case == "k5_uneven_ties":
        K = 5
        sspec = StreamSpec(team_size=K, seed=4, p_uneven=0.5, p_tie=0.5)
    rec = make_stream(sspec, M, P, K=K)
    host = make_roster(rspec)
    dev = make_roster(rspec, device=gpu_device)
    rh = R.BatchRater(host_fp64=True).rate(host, rec, K)
    rd = R.BatchRater().rate(dev, rec.to(gpu_device), K)
    assert torch.equal(rd.status.cpu(), rh.status)
    assert_close_to_fp64(rd, dev, rh, host)


def _exact_dp_device(rank, size, P, M, K, seed):
    from analyzer_amd.parallel.exact_dp import rate_exact_dp

    dev = torch.device("cuda:0")
    roster = make_roster(RosterSpec(num_players=P, seed=seed), device=dev)
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1, p_afk=0.05, p_tie=0.05), M, P, K=K, device=dev)
    out = rate_exact_dp(R.BatchRater(), roster, rec, K)
    return {"state": roster.state.cpu(), "status": out.status.cpu(), "s_mu": out.s_mu.cpu(),
            "delta": out.delta.cpu(), "m_mu": out.m_mu.cpu()}


def test_exact_dp_two_ranks_on_device_bit_identical(gpu_device, tmp_path):
    """C2 on the device: 2 ranks (gloo, both on this GPU) rate a window round by
    round and exchange packed rows; replicas and sharded outputs equal one
    device rating the window alone, bit for bit."""
    from test_distributed import run_ranks

    P, M, K, seed = 3000, 20000, 3, 17
    res = run_ranks(_exact_dp_device, 2, tmp_path, P, M, K, seed)
    roster = make_roster(RosterSpec(num_players=P, seed=seed), device=gpu_device)
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1, p_afk=0.05, p_tie=0.05), M, P, K=K,
                      device=gpu_device)
    ref = R.BatchRater().rate(roster, rec, K)
    want = roster.state.cpu()
    for r in res:
        # tag words of exchanged rows are reset; compare the rating floats
        got, exp = r["state"].view(P, 8, 4), want.view(P, 8, 4)
        for c in (0, 2):
            assert torch.equal(got[..., c].nan_to_num(-7), exp[..., c].nan_to_num(-7))
    owner = torch.stack([r["status"] != 255 for r in res]).sum(0)
    assert bool((owner == 1).all())
    for key in ("s_mu", "delta", "m_mu"):
        merged = torch.full_like(getattr(ref, key).cpu(), float("nan"))
        for r in res:
            mine = r["status"] != 255
            merged[mine] = r[key][mine]
        assert torch.equal(merged.nan_to_num(-7), getattr(ref, key).cpu().nan_to_num(-7)), key


def _rccl_single_rank(rank, size, P, M, K, seed):
    """One RCCL rank on the device: the collectives the DP paths issue, and the
    bucketed sweep merge run through a real (1-rank) RCCL communicator."""
    from analyzer_amd.parallel.comm import all_reduce_sum, all_to_all_rows, world
    from analyzer_amd.parallel.sweep import SweepMerger

    assert torch.distributed.get_backend() == "nccl" and world() == (0, 1)
    dev = torch.device("cuda:0")
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    all_reduce_sum(x)
    y = torch.arange(256, dtype=torch.bfloat16, device=dev).view(64, 4)
    z = torch.empty_like(y)
    all_to_all_rows(z, y)
    g = torch.empty(2000, device=dev)
    torch.distributed.all_gather_into_tensor(g[:1000], x)
    roster = make_roster(RosterSpec(num_players=P, seed=seed), device=dev)
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1), M, P, K=K, device=dev)
    # world_size=2 forces the full merge (messages -> RCCL all-reduce -> decode) on the 1-rank group
    merger = SweepMerger(P, dev, world_size=2, bucket_rows=P // 3 + 1)
    merger.begin(roster)
    R.BatchRater().rate(roster, rec, K)
    posterior = roster.state.clone()
    # the bench's N > 1 defaults: bf16 (fp16 for config 5) messages + int32 touch counts, two
    # collectives per bucket, with the next window's work enqueued while they are in flight
    half = {}
    for cd in ("bf16", "fp16"):
        rh = roster.clone()
        mh = SweepMerger(P, dev, world_size=2, bucket_rows=P // 3 + 1, comm_dtype=cd)
        mh.start.copy_(merger.start)  # the same window start (the pre-rating roster)
        mh._synced = True
        mh.begin(rh)
        half[cd] = (rh, mh)
    # the corrected merge (bench N >= 4): the scan collective (byte rows: bf16 messages +
    # int32 touch fields) on a side stream, the records pass deferred into the next merge
    rc = roster.clone()
    mc = SweepMerger(P, dev, world_size=2, comm_dtype="bf16", correct_records=True, bucket_rows=P // 3 + 1)
    mc.corr_buckets = True
    assert len(mc.buckets()) == 3  # the scan collective per row bucket, on the side stream
    mc.start.copy_(merger.start)
    mc._synced = True
    mc.begin(rc)
    out = R.RateResult.allocate(M, K, dev)
    out.packed.copy_(torch.randn_like(out.packed))
    rows0 = out.packed.clone()
    merger.merge(roster)
    ran = []
    for cd, (rh, mh) in half.items():
        mh.merge(rh, overlap=lambda: ran.append(torch.ones(4, device=dev).sum()))
    mc.merge_corrected(rc, rec, out, overlap=lambda: ran.append(torch.ones(4, device=dev).sum()))
    assert mc._pending is not None  # deferred
    mc.flush_correction()
    mc.check()
    torch.cuda.synchronize()
    assert len(ran) == 3
    return {"x": x.cpu(), "z": z.float().cpu(), "y": y.float().cpu(), "g": g[:1000].cpu(),
            "posterior": posterior.cpu(), "merged": roster.state.cpu(),
            "merged_bf16": half["bf16"][0].state.cpu(), "merged_fp16": half["fp16"][0].state.cpu(),
            "merged_corrected": rc.state.cpu(), "rows_changed": int((out.packed != rows0).sum())}


def test_rccl_single_rank_collectives_and_merge(gpu_device, tmp_path, monkeypatch):
    """RCCL (backend "nccl") on this box: one rank runs the comm layer and the
    pipelined sweep merge through the communicator; with one rank the merge must
    give back the rank's own posterior (up to the natural-parameter round trip).
    Several ranks cannot share one GPU under RCCL -- that path runs in the
    driver's multi-GPU bench."""
    import torch.multiprocessing as mp

    from test_distributed import _free_port

    P, M, K, seed = 5000, 20000, 3, 23
    mp.spawn(_rccl_entry, args=(_free_port(), str(tmp_path), (P, M, K, seed)), nprocs=1, join=True)
    r = torch.load(str(tmp_path / "r0.pt"), weights_only=True)
    assert torch.equal(r["x"], torch.arange(1000, dtype=torch.float32))
    assert torch.equal(r["z"], r["y"]) and torch.equal(r["g"], r["x"])
    post = r["posterior"].view(P, 8, 4)[..., 0::2]
    got = r["merged"].view(P, 8, 4)[..., 0::2]
    np.testing.assert_allclose(got[..., 0].numpy(), post[..., 0].numpy(), rtol=0, atol=2e-3, equal_nan=True)
    np.testing.assert_allclose(got[..., 1].numpy(), post[..., 1].numpy(), rtol=1e-4, atol=0, equal_nan=True)
    # one rank's exclusive prefix is zero: the corrected merge leaves the records alone and
    # decodes like the plain bf16 merge
    assert r["rows_changed"] == 0
    assert torch.equal(r["merged_corrected"].view(torch.int32), r["merged_bf16"].view(torch.int32))
    for cd, tol_mu, tol_sig in (("fp16", 1.0, 2e-3), ("bf16", 8.0, 1e-2)):  # as test_distributed
        gh = r["merged_" + cd].view(P, 8, 4)[..., 0::2]
        np.testing.assert_allclose(gh[..., 0].numpy(), post[..., 0].numpy(), rtol=0, atol=tol_mu, equal_nan=True)
        np.testing.assert_allclose(gh[..., 1].numpy(), post[..., 1].numpy(), rtol=tol_sig, atol=0, equal_nan=True)


def _rccl_entry(rank, port, outdir, args):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        res = _rccl_single_rank(0, 1, *args)
        torch.save(res, os.path.join(outdir, "r0.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,M,K,skew", [(20, 3000, 3, 1), (5000, 100000, 3, 1), (300, 20000, 5, 1),
                                          (100_000, 400_000, 3, 2), (50, 400, 2, 1), (40, 700, 1, 1),
                                          (1_000_000, 1_000_000, 4, 1)])
def test_device_levels_match_host(gpu_device, P, M, K, skew):
    """K5 device levelizer (csrc/levels.hip, a dataflow over the radix or the
    micro-batch schedule) == the sequential host walk, level for level."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.parallel.exact_dp import rounds

    ss = StreamSpec(team_size=K, seed=P + 3, p_afk=0.05, p_unsupported=0.05, p_uneven=0.05, p_hot=0.2,
                    skew=skew)
    rec = make_stream(ss, M, P, K=K)
    lh, dh = native().levels(rec, K, P)
    ld, dd = rounds(rec.to(gpu_device), K, P)
    assert dd == int(dh) and int(lh.max()) == dd
    assert torch.equal(ld, lh)


def test_exact_dp_round_check_on_device(gpu_device):
    """The C2 race detector's kernel (csrc/sweep.hip check_round_kernel) on the
    device: the levelizer's rounds pass, a one-round plan of a window with
    repeated players is flagged -- at the same round as the host path."""
    from analyzer_amd.parallel.exact_dp import RoundPlan, check_rounds, rounds

    P, M, K = 2000, 20000, 3
    rec = make_stream(StreamSpec(team_size=K, seed=5, p_afk=0.05), M, P, K=K, device=gpu_device)
    level, _ = rounds(rec, K, P)
    assert check_rounds(rec, K, RoundPlan(level, 4), P) == -1
    bad = level.clone()
    bad[M // 2:] = bad[M // 2]  # the second half collapses into one round
    plan = RoundPlan(bad, 4)
    assert check_rounds(rec, K, plan, P) == check_rounds(rec.cpu(), K, plan, P) >= 0


def test_make_telemetry_host_counts_match_device(gpu_device, monkeypatch):
    """Worker-sized batches size their synthetic events from host-side counts (no
    device sync); the events equal the device-counted path bit for bit."""
    from analyzer_amd.ops import telemetry as T

    K, P, M = 3, 5000, 1500
    rec = make_stream(StreamSpec(team_size=K, seed=41), M, P, K=K, device=gpu_device)
    spec = T.TelemetrySpec(seed=9, min_events=20, max_events=60)
    a = T.make_telemetry(spec, rec, K, base=1234)
    monkeypatch.setattr(T, "HOST_COUNTS_MAX", 0)
    b = T.make_telemetry(spec, rec, K, base=1234)
    assert torch.equal(a.evoff, b.evoff) and torch.equal(a.events, b.events)


@pytest.mark.parametrize("dtype,N", [(torch.bfloat16, 8), (torch.float16, 8), (torch.bfloat16, 3), (torch.float16, 1)])
def test_split_block_reduce_kernel_matches_host(gpu_device, dtype, N):
    """csrc/sweep.hip sweep_block_reduce (the split merge's owner reduce) against the host
    reduce parallel/comm.py block_reduce_rows, bit for bit: sums and exclusive prefixes of
    the 16-bit halves in fp32 in rank order, rounded once; touch words as integers."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.parallel.comm import block_reduce_rows

    g = torch.Generator().manual_seed(5 + N)
    blk = 10007
    h = (torch.randn((N * blk, 14), generator=g) * 40).to(dtype)
    recv = torch.empty((N * blk, 8), dtype=torch.int32)
    recv[:, :7] = h.view(torch.int32)
    recv[:, 7] = torch.randint(0, 1 << 20, (N * blk,), generator=g, dtype=torch.int32)
    tot_h, pref_h = block_reduce_rows(recv, N, dtype, True)
    rd = recv.to(gpu_device)
    tot = torch.empty((blk, 8), dtype=torch.int32, device=gpu_device)
    pref = torch.empty((N * blk, 7), dtype=torch.int32, device=gpu_device)
    native().sweep_block_reduce(rd, N, dtype == torch.bfloat16, tot, pref)
    tot2 = torch.empty_like(tot)
    native().sweep_block_reduce(rd, N, dtype == torch.bfloat16, tot2)  # no prefix
    torch.cuda.synchronize()
    assert torch.equal(tot.cpu(), tot_h) and torch.equal(tot2.cpu(), tot_h)
    assert torch.equal(pref.cpu(), pref_h)
