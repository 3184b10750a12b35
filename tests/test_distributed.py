"""Multi-process tests of the comm layer on the CPU (gloo, world size 2-4):
C1 sweep merge, C2 exact DP, C3 broadcast, C4 metric reduce.
Each test spawns ranks that write their results to a temp dir; the parent checks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank, size, port, fn, outdir, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(size), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        res = fn(rank, size, *args)
        torch.save(res, os.path.join(outdir, "r%d.pt" % rank))
    finally:
        dist.destroy_process_group()


def run_ranks(fn, size, tmp_path, *args):
    os.makedirs(str(tmp_path), exist_ok=True)
    mp.spawn(_entry, args=(size, _free_port(), fn, str(tmp_path), args), nprocs=size, join=True)
    return [torch.load(os.path.join(str(tmp_path), "r%d.pt" % r), weights_only=True) for r in range(size)]


# ------------------------------------------------------------------ C3 / C4
def _bcast_and_counts(rank, size):
    from analyzer_amd.ops.rate import Roster
    from analyzer_amd.parallel.comm import broadcast_roster, reduce_counts

    roster = make_roster(RosterSpec(num_players=50, seed=4)) if rank == 0 else Roster.empty(50)
    broadcast_roster(roster)
    c = reduce_counts({"rated": 10.0 * (rank + 1), "only_r%d" % rank: 1.0}, "cpu")
    m = reduce_counts({"ms": float(rank)}, "cpu", op="max")
    return {"state": roster.state, "attrs": roster.attrs, "counts": c, "max": m}


def test_broadcast_roster_and_reduce_counts(tmp_path):
    res = run_ranks(_bcast_and_counts, 3, tmp_path)
    ref = make_roster(RosterSpec(num_players=50, seed=4))
    for r in res:
        assert torch.equal(r["state"].nan_to_num(-7), ref.state.nan_to_num(-7))
        assert torch.equal(r["attrs"].nan_to_num(-7), ref.attrs.nan_to_num(-7))
        assert r["counts"] == {"rated": 60.0, "only_r0": 1.0, "only_r1": 1.0, "only_r2": 1.0}
        assert r["max"] == {"ms": 2.0}


# ------------------------------------------------------------------ C2 exact DP
def _exact(rank, size, P, M, K, seed):
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.exact_dp import rate_exact_dp

    roster = make_roster(RosterSpec(num_players=P, seed=seed))
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1, p_afk=0.05, p_unsupported=0.05), M, P, K=K)
    out = rate_exact_dp(BatchRater(), roster, rec, K)
    return {"state": roster.state, "status": out.status.clone(), "s_mu": out.s_mu.clone(),
            "delta": out.delta.clone(), "m_mu": out.m_mu.clone(), "quality": out.quality.clone()}


@pytest.mark.parametrize("size", [2, 3])
def test_exact_dp_bit_identical_to_sequential(tmp_path, size):
    from analyzer_amd.ops.rate import BatchRater

    P, M, K, seed = 40, 300, 3, 9
    res = run_ranks(_exact, size, tmp_path, P, M, K, seed)
    roster = make_roster(RosterSpec(num_players=P, seed=seed))
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1, p_afk=0.05, p_unsupported=0.05), M, P, K=K)
    ref = BatchRater().rate(roster, rec, K)
    for r in res:  # replicas agree with the sequential run, bit for bit
        assert torch.equal(r["state"].nan_to_num(-7), roster.state.nan_to_num(-7))
    # outputs are sharded: every match rated by exactly one rank, identical values
    owner = torch.stack([r["status"] != 255 for r in res]).sum(0)
    assert bool((owner == 1).all())
    for key, ref_t in (("s_mu", ref.s_mu), ("delta", ref.delta), ("m_mu", ref.m_mu)):
        merged = torch.full_like(ref_t, float("nan"))
        for r in res:
            mine = r["status"] != 255
            merged[mine] = r[key][mine]
        assert torch.equal(merged.nan_to_num(-7), ref_t.nan_to_num(-7)), key


def test_levels_host():
    from analyzer_amd.ops.native import native

    rec = make_stream(StreamSpec(team_size=3, seed=2, p_afk=0.0), 200, 15)
    level, depth = native().levels(rec, 3, 15)
    last = {}
    for m in range(200):
        ids = [int(x) for x in rec[m, :6]]
        exp = 1 + max(last.get(p, 0) for p in ids)
        assert int(level[m]) == exp
        for p in ids:
            last[p] = exp
    assert depth == int(level.max())


# ------------------------------------------------------------------ C1 sweep merge
def _sweep(rank, size, P, M, K, seed, disjoint, comm_dtype="fp32"):
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.sweep import SweepMerger

    roster = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.5))
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1 + rank, p_afk=0.0), M, P, K=K)
    if disjoint:  # rank r only sees players r, r+size, ...
        rec[:, :2 * K] = rec[:, :2 * K] - rec[:, :2 * K] % size + rank
    merger = SweepMerger(P, "cpu", comm_dtype=comm_dtype)
    merger.begin(roster)
    local = roster.clone()
    BatchRater().rate(local, rec, K)
    merger.messages(local)
    msg = merger.buf.clone()
    merger.reduce()
    merged = local.clone()
    merger.apply(merged)
    return {"local": local.state, "msg": msg, "merged": merged.state, "rec": rec}


def test_sweep_merge_disjoint_equals_union(tmp_path):
    """Players partitioned across ranks: the merge reproduces every rank's exact
    result (up to the natural-parameter round trip in fp32)."""
    P, M, K, seed, size = 60, 200, 3, 5, 2
    res = run_ranks(_sweep, size, tmp_path, P, M, K, seed, True)
    for rank, r in enumerate(res):
        mine = torch.arange(P) % size == rank
        a, b = r["merged"][mine], r["local"][mine]
        mu_a, mu_b = a[:, 0::4], b[:, 0::4]
        assert torch.equal(torch.isnan(mu_a), torch.isnan(mu_b))
        ok = ~torch.isnan(mu_b)
        assert torch.allclose(mu_a[ok], mu_b[ok], rtol=1e-5, atol=2e-3)
        sg_a, sg_b = a[:, 2::4][ok], b[:, 2::4][ok]
        assert torch.allclose(sg_a, sg_b, rtol=1e-4)
    assert torch.equal(res[0]["merged"].nan_to_num(-7), res[1]["merged"].nan_to_num(-7))


def _merged_ratio(S, m):
    """sweep_core.h merged_ratio, re-derived: (pi / pi_B, mean-shift divisor)."""
    var = (S < 0) & (m >= 2)
    x = 1 + S / m.clamp(min=1)
    return torch.where(var, x / (x + m * (1 - x)), 1 + S), torch.where(var, x, 1 + S), var


def test_sweep_merge_overlapping_sums_messages(tmp_path):
    """Overlapping players: merged natural parameters = start + sum of every
    rank's (posterior - start) message (EP product of the rank posteriors) where the
    ranks net-gained precision; a net loss (tau^2 dynamics) over m >= 2 ranks is
    combined in variance space (sweep_core.h merged_ratio)."""
    P, M, K, seed, size = 30, 150, 3, 6, 3
    res = run_ranks(_sweep, size, tmp_path, P, M, K, seed, False)
    total = sum(r["msg"] for r in res)
    start = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.5)).state
    merged = res[0]["merged"]
    lo, hi = total[:, 14].long(), total[:, 15].long()
    n_var = 0
    for t in range(7):
        m = (lo >> (4 * t)) & 15 if t < 4 else (hi >> (4 * (t - 4))) & 15
        mu0, sg0 = start[:, 4 * t], start[:, 4 * t + 2]
        have = ~torch.isnan(mu0) & ((total[:, 2 * t] != 0) | (total[:, 2 * t + 1] != 0))
        pb = 1 / sg0[have].double() ** 2
        mb = mu0[have].double()
        dpi, dtau = total[have, 2 * t].double(), total[have, 2 * t + 1].double()
        ratio, mdiv, var = _merged_ratio(dpi / pb, m[have].double())
        mu = torch.where(var, mb + (dtau / pb - dpi / pb * mb) / mdiv, (mb * pb + dtau) / (pb + dpi))
        assert torch.allclose(merged[have, 4 * t].double(), mu, rtol=1e-5, atol=1e-2)
        assert torch.allclose(merged[have, 4 * t + 2].double(), (pb * ratio).rsqrt(), rtol=1e-4)
        n_var += int(var.sum())
    assert n_var > 0  # both branches exercised
    for r in res[1:]:
        assert torch.equal(r["merged"].nan_to_num(-7), merged.nan_to_num(-7))


def _sweep_buckets(rank, size, P, M, K, seed, comm_dtype, bucket_rows):
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.sweep import SweepMerger

    roster = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.5))
    rec = make_stream(StreamSpec(team_size=K, seed=seed + 1 + rank, p_afk=0.0), M, P, K=K)
    out = {}
    for rows, tag in ((None, "whole"), (bucket_rows, "bucketed"), (bucket_rows, "overlap")):
        merger = SweepMerger(P, "cpu", comm_dtype=comm_dtype,
                             bucket_rows=P if rows is None else rows)
        local = roster.clone()
        merger.begin(local)
        BatchRater().rate(local, rec, K)
        calls = []
        # "overlap": all buckets' all-reduces launched, the overlapped work, then the decodes
        merger.merge(local, overlap=(lambda: calls.append(1)) if tag == "overlap" else None)
        out[tag] = local.state
        out["n_buckets_%s" % tag] = len(merger.buckets())
        out["calls_%s" % tag] = len(calls)
    return out


@pytest.mark.parametrize("comm_dtype", ["fp32", "fp16", "bf16"])
def test_sweep_merge_bucketed_pipeline_matches_single_bucket(tmp_path, comm_dtype):
    """The pipelined merge (messages / async all-reduce / apply per row bucket,
    ragged last bucket) gives the one-bucket result bit for bit: every stage is
    per player, and two-rank sums do not depend on the reduction order."""
    P, M, K, seed, size = 101, 300, 3, 9, 2
    res = run_ranks(_sweep_buckets, size, tmp_path, P, M, K, seed, comm_dtype, 16)
    for r in res:
        assert r["n_buckets_whole"] == 1 and r["n_buckets_bucketed"] == 7
        assert torch.equal(r["whole"].nan_to_num(-7), r["bucketed"].nan_to_num(-7))
        assert r["calls_overlap"] == 1 and r["calls_bucketed"] == 0
        assert torch.equal(r["whole"].nan_to_num(-7), r["overlap"].nan_to_num(-7))
    assert torch.equal(res[0]["bucketed"].nan_to_num(-7), res[1]["bucketed"].nan_to_num(-7))


@pytest.mark.parametrize("dtype,tol_mu", [("fp16", 1.0), ("bf16", 8.0)])
def test_sweep_merge_compressed_messages(tmp_path, dtype, tol_mu):
    """COMM_DTYPE fp16/bf16: base-relative messages survive the compressed
    all-reduce (config 5 "fp16 moments"); merged ratings stay close to fp32."""
    P, M, K, seed, size = 200, 600, 3, 7, 2
    ref = run_ranks(_sweep, size, tmp_path / "a", P, M, K, seed, False, "fp32")
    got = run_ranks(_sweep, size, tmp_path / "b", P, M, K, seed, False, dtype)
    a, b = ref[0]["merged"], got[0]["merged"]
    mu_a, mu_b = a[:, 0::4], b[:, 0::4]
    assert torch.equal(torch.isnan(mu_a), torch.isnan(mu_b))
    ok = ~torch.isnan(mu_a)
    err = (mu_a[ok] - mu_b[ok]).abs()
    # rating shifts of hundreds of points per window: fp16 keeps ~5e-4 of them, bf16 ~4e-3
    assert float(err.max()) < tol_mu and float(err.median()) < tol_mu / 10
    sg_a, sg_b = a[:, 2::4][ok], b[:, 2::4][ok]
    assert float(((sg_a - sg_b).abs() / sg_a).max()) < 2e-2
    assert torch.equal(got[0]["merged"].nan_to_num(-7), got[1]["merged"].nan_to_num(-7))


# ------------------------------------------------ causal re-sweeps (K9 + C1')
def _scan(rank, size):
    from analyzer_amd.parallel.comm import exclusive_scan

    t = torch.arange(7 * 3, dtype=torch.float32).view(7, 3) * (rank + 1)
    return {"ex": exclusive_scan(t)}


def test_exclusive_scan_over_ranks(tmp_path):
    size = 3
    res = run_ranks(_scan, size, tmp_path)
    base = torch.arange(7 * 3, dtype=torch.float32).view(7, 3)
    for r, out in enumerate(res):
        assert torch.equal(out["ex"], base * sum(q + 1 for q in range(r)))


def _resweep(rank, size, P, M, K, seed, sweeps, comm_dtype):
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.sweep import SweepMerger, rate_window_dp

    roster = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.3))
    spec = StreamSpec(team_size=K, seed=seed + 1)
    merger = SweepMerger(P, "cpu", comm_dtype=comm_dtype, sweeps=sweeps)
    outs = []
    for w in range(2):  # two windows: the second starts from the merge's own start copy
        rec = make_stream(spec, M, P, K=K, base=(w * size + rank) * M)
        outs.append(rate_window_dp(BatchRater(), merger, roster, rec, K).s_mu.clone())
    return {"state": roster.state, "s_mu": outs[-1]}


@pytest.mark.parametrize("sweeps", [1, 2, 3])
def test_causal_resweeps_converge_to_exact(tmp_path, sweeps):
    """N gloo ranks rate consecutive time slices; ``sweeps`` causal re-sweeps
    (exclusive prefix of the earlier ranks' messages) converge to the exact
    sequential result: at sweeps == N it is reproduced up to fp32 rounding, and
    the distributed run equals the one-process simulation (parallel/accuracy.py)."""
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.accuracy import compare, simulate_sweep_dp

    P, M, K, seed, size = 300, 700, 3, 21, 3
    res = run_ranks(_resweep, size, tmp_path, P, M, K, seed, sweeps, "fp32")
    spec = StreamSpec(team_size=K, seed=seed + 1)
    start = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.3))
    exact, sim = start.clone(), start.clone()
    for w in range(2):
        shards = [make_stream(spec, M, P, K=K, base=(w * size + r) * M) for r in range(size)]
        ref_out = [BatchRater().rate(exact, sh, K) for sh in shards]
        simulate_sweep_dp(BatchRater(), sim, shards, K, sweeps=sweeps)
    for r in res[1:]:  # replicas agree
        assert torch.equal(r["state"].nan_to_num(-7), res[0]["state"].nan_to_num(-7))
    got = res[0]["state"]
    # distributed == simulation (sums of 3 fp32 messages may round differently)
    ok = ~torch.isnan(sim.state[:, 0::4])
    assert torch.equal(torch.isnan(got[:, 0::4]), ~ok)
    assert float((got[:, 0::4][ok] - sim.state[:, 0::4][ok]).abs().max()) < 1e-2
    from analyzer_amd.ops.rate import Roster

    stats = compare(Roster(got, start.attrs), exact)
    sh = stats["tracks"]["shared"]
    assert sh["null_mismatch"] == 0
    bound = {1: None, 2: None, 3: 0.02}[sweeps]
    if bound is not None:
        assert sh["dmu_max"] < bound, sh
        # the last rank's records are exact too
        last = ref_out[-1].s_mu
        d = (res[-1]["s_mu"] - last).abs()
        assert float(d[~torch.isnan(d)].max()) < bound


def test_resweep_error_falls_per_sweep():
    """One-process simulation, 4 ranks: each causal re-sweep cuts the deviation
    from exact by more than 5x, and sweeps == ranks is exact to fp32 rounding."""
    from analyzer_amd.parallel.accuracy import run

    t = run(ranks=4, players=1500, matches_per_rank=3000, windows=2, sweeps=[1, 2, 3, 4],
            warm_windows=1)
    errs = [t["sweeps"][str(s)]["tracks"]["shared"] for s in (1, 2, 3, 4)]
    for a, b in zip(errs, errs[1:]):
        assert b["dmu_p99"] < a["dmu_p99"] / 5, (a, b)
    assert errs[-1]["dmu_max"] < 5e-3
    assert errs[0]["dmu_median"] > 1.0  # one sweep is a real approximation at this density
    for e in errs:
        assert e["null_mismatch"] == 0
    assert t["sweeps"]["4"]["records_shared_mu"]["dmu_max"] < 5e-3


def test_round_check_flags_shared_players():
    """C2 race detector (ANA_CHECK_ROUNDS): the levelizer's rounds pass; a plan
    that puts a player's two consecutive matches in one round is caught."""
    import numpy as np

    from analyzer_amd.parallel.exact_dp import RoundPlan, check_rounds, rounds

    P, M, K = 60, 400, 3
    rec = make_stream(StreamSpec(team_size=K, seed=3, p_afk=0.05, p_unsupported=0.05), M, P, K=K)
    level, _ = rounds(rec, K, P)
    assert check_rounds(rec, K, RoundPlan(level, 2), P) == -1
    bad = level.clone()
    bad[:] = 1  # everything in one round: players repeat
    assert check_rounds(rec, K, RoundPlan(bad, 2), P) == 0


def _exact_checked(rank, size, P, M, K, seed):
    import os

    os.environ["ANA_CHECK_ROUNDS"] = "1"
    return _exact(rank, size, P, M, K, seed)


def test_exact_dp_with_round_check(tmp_path):
    res = run_ranks(_exact_checked, 2, tmp_path, 40, 300, 3, 9)
    assert len(res) == 2


def _probe(rank, size):
    from analyzer_amd.parallel.comm import time_all_reduce

    t = torch.ones(1 << 16) * (rank + 1)
    ms = time_all_reduce(t)
    return {"ms": torch.tensor([ms], dtype=torch.float64)}


def test_all_reduce_probe_agrees_across_ranks(tmp_path):
    """The DP placement probe (runtime/engine.py probe_placement) times a merge-sized
    all-reduce; every rank gets the same (max) time, so every rank takes the same
    prepass placement."""
    res = run_ranks(_probe, 3, tmp_path)
    assert float(res[0]["ms"]) > 0.0
    for r in res[1:]:
        assert torch.equal(r["ms"], res[0]["ms"])


# ------------------------------------------------ merge decodes fail loudly
def test_decode_clamps_are_counted_and_raise():
    """A summed message that drives a track's merged precision to or below zero is
    held at the floor by the decode -- and counted, host mirror and merger alike:
    SweepMerger.check raises MergeClampError instead of writing sigma x1000 silently
    (the reference raises on numeric trouble and dead-letters the batch,
    /root/reference/rater.py:7-8, worker.py:108-120)."""
    from analyzer_amd.ops.native import native
    from analyzer_amd.ops.synth import RosterSpec, make_roster
    from analyzer_amd.parallel.sweep import MergeClampError, SweepMerger, base_rows

    P = 64
    ro = make_roster(RosterSpec(num_players=P, seed=3, p_rated=1.0, p_mode_rated=1.0))
    for comm in ("fp32", "bf16"):
        m = SweepMerger(P, "cpu", comm_dtype=comm, force=True)
        m.begin(ro.clone())
        if comm == "fp32":  # raw (d_pi, d_tau): a precision loss larger than the base's
            m.buf.zero_()
            pi = 1.0 / m.start[:5, 1] ** 2
            m.buf[:5, 0] = -2.0 * pi
            m.decode(ro.clone())
        else:               # scaled: 1 + sum r_pi <= 0 on the shared track of 5 players
            m.msg.zero_()
            m.cnt.zero_()
            m.msg[:5, 0] = -1.5
            m.decode_packed(ro.clone())
        assert m.clamp_hits() == 5
        with pytest.raises(MergeClampError, match="5 decoded track"):
            m.check()
        assert m.clamp_hits() == 0  # restarted
        m.check()
    # the plain decode of a healthy sum clamps nothing
    m = SweepMerger(P, "cpu", comm_dtype="bf16", force=True)
    r2 = ro.clone()
    m.begin(r2)
    m.messages_packed(r2)
    m.decode_packed(r2)
    m.check()
    assert torch.equal(base_rows(r2.state).nan_to_num(-7), base_rows(ro.state).nan_to_num(-7))


def test_net_precision_loss_over_ranks_decodes_in_variance_space():
    """Eight ranks that each lost 20 % of a track's precision to tau^2 dynamics (a
    low-sigma player in every slice -- the 1M-player 8-rank bench hit 28 such tracks):
    the natural-parameter sum is 1 - 1.6 < 0, the decode combines the losses in
    variance space instead -- 1 / (1 + 8 (1 / 0.8 - 1)) = 1/3 of the precision, what
    sequential dynamics give -- and clamps nothing; one rank's loss stays exact."""
    from analyzer_amd.ops.synth import RosterSpec, make_roster
    from analyzer_amd.parallel.sweep import SweepMerger

    P = 16
    ro = make_roster(RosterSpec(num_players=P, seed=3, p_rated=1.0, p_mode_rated=1.0))
    for comm in ("bf16", "fp32"):
        for m_ranks, S, want in ((8, -1.6, 1.0 / 3.0), (1, -0.7, 0.3)):
            mg = SweepMerger(P, "cpu", comm_dtype=comm, force=True)
            r = ro.clone()
            mg.begin(r)
            sg0 = mg.start[:, 1].double()
            if comm == "bf16":
                mg.msg.zero_()
                mg.cnt.zero_()
                mg.msg[:, 0] = S
                mg.cnt[:, 0] = m_ranks  # shared track: touch field 0
                mg.decode_packed(r)
            else:
                mg.buf.zero_()
                mg.buf[:, 0] = (S / sg0 ** 2).float()
                mg.buf[:, 1] = mg.buf[:, 0] * mg.start[:, 0]  # d_tau of an unmoved mean: mu_B d_pi
                mg.buf[:, 14] = float(m_ranks)
                mg.decode(r)
            assert mg.clamp_hits() == 0
            got = (sg0 / r.state[:, 2].double()) ** 2  # pi / pi_B
            assert torch.allclose(got, torch.full_like(got, want), rtol=2e-2), (comm, m_ranks, got[:3])
            mu_shift = (r.state[:, 0].double() - mg.start[:, 0].double()).abs()
            assert float(mu_shift.max()) < 1e-2  # no mean message: the mean stays


def test_default_merge_keeps_its_precision_margin_at_the_lag_reproduction_density():
    """The round-4 lagged merge diverged at 8 ranks x 125k matches per rank-window over
    100k players (profiles/r5/lag_bf16_root_cause.log: messages measured against each
    rank's own start overshoot the common precision, 1 + sum r_pi crosses zero).  The
    merge that remains measures every rank against the common start: at the same
    density (8 ranks, 7.5 appearances per player per rank-window, bf16 messages, three
    windows from a warm roster) no decode clamps and the roster stays close."""
    from analyzer_amd.parallel.accuracy import run

    t = run(ranks=8, players=8_000, matches_per_rank=10_000, windows=3, sweeps=[1], comm_dtype="bf16",
            warm_windows=1)
    st = t["sweeps"]["1"]
    assert st["clamp_hits"] == 0
    sh = st["tracks"]["shared"]
    assert sh["spearman_mu_minus_sigma"] > 0.99 and sh["dmu_max"] < 1000.0, sh


# ------------------------------------------------ causal record correction
def _scan_sum(rank, size):
    from analyzer_amd.parallel.comm import scan_and_sum

    t = (torch.arange(22 * 5, dtype=torch.float32).view(22, 5) + 100 * rank).to(torch.bfloat16)
    c = torch.full((22, 2), rank + 1, dtype=torch.int32)
    p, s = scan_and_sum(t)
    pc, sc = scan_and_sum(c)
    from analyzer_amd.parallel.comm import scan_and_sum_rows

    p2, s2, e2 = scan_and_sum_rows(t, c.clone())  # one payload: bf16 rows + int32 rows
    return {"p": p.float(), "s": s.float(), "pc": pc, "sc": sc, "p2": p2.float(), "s2": s2.float(), "e2": e2}


def test_scan_and_sum_over_ranks(tmp_path):
    """One exchange gives every rank the sum over ranks and its exclusive prefix
    (ragged row blocks, bf16 summed in fp32 and rounded once, int32 exact)."""
    size = 3
    res = run_ranks(_scan_sum, size, tmp_path)
    ts = [(torch.arange(22 * 5, dtype=torch.float32).view(22, 5) + 100 * r).to(torch.bfloat16).float()
          for r in range(size)]
    for r, out in enumerate(res):
        exp_p = sum(ts[:r], torch.zeros(22, 5)).to(torch.bfloat16).float()
        assert torch.equal(out["p"], exp_p)
        assert torch.equal(out["s"], sum(ts).to(torch.bfloat16).float())
        assert torch.equal(out["pc"], torch.full((22, 2), sum(range(1, r + 1)), dtype=torch.int32))
        assert torch.equal(out["sc"], torch.full((22, 2), 6, dtype=torch.int32))
        assert torch.equal(out["p2"], out["p"]) and torch.equal(out["s2"], out["s"])
        assert torch.equal(out["e2"], out["sc"])


def _corrected(rank, size, P, M, K, seed, windows, comm_dtype):
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.sweep import SweepMerger
    from analyzer_amd.runtime.engine import WindowPipeline

    roster = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.3))
    spec = StreamSpec(team_size=K, seed=seed + 1)
    recs = [make_stream(spec, M, P, K=K, base=(w * size + rank) * M) for w in range(windows)]
    merger = SweepMerger(P, "cpu", comm_dtype=comm_dtype)
    pipe = WindowPipeline(BatchRater(), roster, K, merger=merger)
    outs = []
    pipe.run(recs, on_result=lambda i, res: outs.append((res.s_mu.clone(), res.m_mu.clone())))
    return {"state": roster.state, "last": outs[-1]}


def _corrected_ring(rank, size, P, M, K, seed, windows, mode):
    """bench.py's use: windows rated into two alternating record buffers, nothing
    consumed until finish().  mode: "split" (the round-6 merge: the sum on the critical
    path, prefix + correction deferred), "defer" / "inline" (the round-5 scan merge with
    the correction run inside the next merge / right after the decode)."""
    import os

    from analyzer_amd.ops.rate import BatchRater, RateResult
    from analyzer_amd.parallel.sweep import SweepMerger
    from analyzer_amd.runtime.engine import WindowPipeline

    os.environ["ANA_DP_SPLIT"] = "1" if mode == "split" else "0"
    os.environ["ANA_DP_CORRECT_DEFER"] = "1" if mode in ("defer", "bucketed") else "0"
    os.environ["ANA_DP_CORR_BUCKETS"] = "1" if mode == "bucketed" else "0"
    roster = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.3))
    spec = StreamSpec(team_size=K, seed=seed + 1)
    recs = [make_stream(spec, M, P, K=K, base=(w * size + rank) * M) for w in range(windows)]
    # "bucketed": the scan merge pipelined over 4 row buckets (a ragged last one)
    merger = SweepMerger(P, "cpu", comm_dtype="bf16", correct_records=True,
                         bucket_rows=P // 4 + 1 if mode == "bucketed" else None)
    assert len(merger.buckets()) == (4 if mode == "bucketed" else 1)
    assert merger.split() == (mode == "split"), (mode, merger.split())
    pipe = WindowPipeline(BatchRater(), roster, K, merger=merger)
    outs = [RateResult.allocate(M, K, "cpu") for _ in range(2)]
    prep = pipe.prepare(recs[0])
    for w in range(windows):
        _, prep = pipe.step(prep, recs[w + 1] if w + 1 < windows else None, out=outs[w % 2])
    pending = merger._pending is not None
    pipe.finish()
    return {"rows": [o.packed.clone() for o in outs], "pending": pending, "state": roster.state}


def test_deferred_record_correction_matches_inline(tmp_path):
    """The record correction deferred into the next merge (beside its collective), the
    same merge pipelined over row buckets, and the round-6 split merge (all-to-all /
    owner reduce / all-gather of the sum, the prefix returned and the records corrected
    after the decode), write exactly the records and the roster the in-line pass writes,
    once finish() has run."""
    P, M, K, seed, size, windows = 300, 700, 3, 41, 2, 3
    a = run_ranks(_corrected_ring, size, tmp_path, P, M, K, seed, windows, "defer")
    b = run_ranks(_corrected_ring, size, tmp_path, P, M, K, seed, windows, "inline")
    c = run_ranks(_corrected_ring, size, tmp_path, P, M, K, seed, windows, "split")
    d = run_ranks(_corrected_ring, size, tmp_path, P, M, K, seed, windows, "bucketed")
    for r in range(size):
        assert a[r]["pending"] and not b[r]["pending"] and d[r]["pending"]
        for o in (a[r], c[r], d[r]):
            assert torch.equal(o["state"].view(torch.int32), b[r]["state"].view(torch.int32))
            for x, y in zip(o["rows"], b[r]["rows"]):
                assert torch.equal(x.view(torch.int32), y.view(torch.int32))


@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_record_correction_over_ranks_equals_simulation(tmp_path, comm_dtype):
    """The corrected merge over gloo (scan_and_sum, the records pass before the
    decode) gives every rank's records what the one-process simulation of
    parallel/accuracy.py gives, and the corrected records sit much closer to exact
    sequential rating than the uncorrected ones."""
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.accuracy import compare, simulate_sweep_dp

    P, M, K, seed, size, windows = 400, 900, 3, 31, 3, 3
    res = run_ranks(_corrected, size, tmp_path, P, M, K, seed, windows, comm_dtype)
    spec = StreamSpec(team_size=K, seed=seed + 1)
    sets = [[make_stream(spec, M, P, K=K, base=(w * size + r) * M) for r in range(size)] for w in range(windows)]
    start = make_roster(RosterSpec(num_players=P, seed=seed, p_rated=0.3))
    tol = 1e-3 if comm_dtype == "fp32" else 0.2
    for correct in (True, False):
        sim = start.clone()
        for shards in sets:
            outs = simulate_sweep_dp(BatchRater(), sim, shards, K, comm_dtype=comm_dtype, correct=correct)
        if correct:
            for r in range(size):
                for got, exp in zip(res[r]["last"], (outs[r].s_mu, outs[r].m_mu)):
                    d = (got - exp).abs()
                    assert torch.equal(torch.isnan(got), torch.isnan(exp))
                    assert float(d[~torch.isnan(d)].max()) < tol
            assert torch.equal(torch.isnan(res[0]["state"]), torch.isnan(sim.state))
            corrected = outs
        else:
            plain = outs
    exact = start.clone()
    out_e = None
    for shards in sets:
        out_e = [BatchRater().rate(exact, sh, K) for sh in shards]
    med_c = compare(sim, exact, corrected, out_e)["records_shared_mu"]["dmu_median"]
    med_p = compare(sim, exact, plain, out_e)["records_shared_mu"]["dmu_median"]
    assert med_c < 0.6 * med_p, (med_c, med_p)


def test_packed_touch_word_decodes_like_the_fp32_fields():
    """The compressed merge carries the two base-16 touch fields in one int32 (lo | hi << 16:
    tracks 0-3 in lo, 4-6 in hi).  On the host path, the packed decode of a sum with touch
    counts on every track -- mode tracks (hi) included -- equals the fp32 decode of the same
    fields, and the packed messages round-trip the fields exactly."""
    from analyzer_amd.models.tiers import vst_table
    from analyzer_amd.ops.native import native
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.parallel.sweep import base_rows

    P = 3000
    start = make_roster(RosterSpec(num_players=P, seed=5, p_rated=0.7))
    after = start.clone()
    BatchRater().rate(after, make_stream(StreamSpec(team_size=3, seed=6), 12000, P), 3)
    vst = torch.tensor(vst_table(), dtype=torch.float32)
    sb = base_rows(start.state).contiguous()
    buf = torch.empty((P, 16))
    native().sweep_delta(sb, sb, after.state, start.attrs, vst, 500.0, True, buf)
    msg = torch.empty((P, 14), dtype=torch.bfloat16)
    cnt = torch.empty((P, 1), dtype=torch.int32)
    native().sweep_delta_packed(sb, sb, after.state, start.attrs, vst, 500.0, msg, cnt)
    lohi = buf[:, 14:].to(torch.int32)
    assert torch.equal(cnt, lohi[:, :1] | (lohi[:, 1:] << 16))
    assert int((lohi[:, 1] > 0).sum()) > 0, "some mode track (hi field) must be touched"
    # a "sum" over three ranks: every nibble x3 (no carry below 16)
    msg3, cnt3 = (msg.float() * 3).to(torch.bfloat16), cnt * 3
    joined = torch.cat([msg3.float(), (cnt3 & 0xffff).float(), (cnt3 >> 16).float()], dim=1)
    s_ref, s2_ref = start.state.clone(), torch.zeros_like(sb)
    native().sweep_apply(sb, joined, start.attrs, s_ref, s2_ref, vst, 500.0, True)
    s_p, s2_p = start.state.clone(), torch.zeros_like(sb)
    native().sweep_apply_packed(sb, msg3, cnt3, start.attrs, s_p, s2_p, vst, 500.0)
    assert torch.equal(s_p.nan_to_num(-7), s_ref.nan_to_num(-7))
    assert torch.equal(s2_p.nan_to_num(-7), s2_ref.nan_to_num(-7))


def _split_ex(rank, size):
    from analyzer_amd.parallel.comm import SplitExchange

    P = 22
    h = (torch.arange(P * 14, dtype=torch.float32).view(P, 14) * 0.37 + 100 * rank).to(torch.bfloat16)
    op = torch.empty((P, 8), dtype=torch.int32)
    op[:, :7] = h.view(torch.int32)
    op[:, 7] = rank + 1
    ex = SplitExchange(op, torch.bfloat16, want_prefix=True)
    return {"h": h.float(), "total": ex.total().clone(), "prefix": ex.prefix().clone()}


def test_split_exchange_over_ranks(tmp_path):
    """The split merge's collective (comm.SplitExchange): every rank gets the sum over
    ranks (bf16 summed in fp32 in rank order, rounded once; the touch word as an integer)
    and its exclusive prefix, with ragged row blocks (22 rows over 3 ranks)."""
    size = 3
    res = run_ranks(_split_ex, size, tmp_path)
    hs = [r["h"] for r in res]
    for r, out in enumerate(res):
        acc = torch.zeros(22, 14)
        for q in range(r):
            acc = acc + hs[q]
        assert torch.equal(out["prefix"].view(torch.bfloat16).float(), acc.to(torch.bfloat16).float())
        tot = torch.zeros(22, 14)
        for q in range(size):
            tot = tot + hs[q]
        assert torch.equal(out["total"][:, :7].contiguous().view(torch.bfloat16).float(),
                           tot.to(torch.bfloat16).float())
        assert torch.equal(out["total"][:, 7], torch.full((22,), 6, dtype=torch.int32))


def test_reused_records_tensor_is_refused():
    """A window whose records tensor is the previous window's (refilled in place) is
    refused while that window's record correction is still deferred: the correction
    would read the new window's player ids (advisor finding, round 5)."""
    from analyzer_amd.ops.rate import BatchRater, RateResult
    from analyzer_amd.parallel.sweep import SweepMerger
    from analyzer_amd.runtime.engine import WindowPipeline

    P, M, K = 200, 300, 3
    roster = make_roster(RosterSpec(num_players=P, seed=3))
    rec = make_stream(StreamSpec(team_size=K, seed=4), M, P, K=K)
    merger = SweepMerger(P, "cpu", comm_dtype="bf16", correct_records=True, world_size=1, force=True)
    merger.defer = True
    pipe = WindowPipeline(BatchRater(), roster, K, merger=merger)
    out = [RateResult.allocate(M, K, "cpu") for _ in range(2)]
    prep = pipe.prepare(rec)
    _, prep2 = pipe.step(prep, rec, out=out[0])  # the next window reuses the same tensor
    assert merger.rec_in_use(rec)
    with pytest.raises(ValueError):
        pipe.step(prep2, None, out=out[1])
