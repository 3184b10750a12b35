"""Full-history re-rate driver, checkpoint/resume and fault injection (SURVEY
P4, C5, §4 item 6) on the CPU (host mirror; gloo for the multi-rank case)."""
import os

import pytest
import torch

from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import make_roster, make_stream
from analyzer_amd.runtime import checkpoint
from analyzer_amd.runtime.rerate import InjectedFault, RerateSpec, run

from test_distributed import run_ranks

SPEC = RerateSpec(total_matches=1250, players=80, team_size=3, window=300, seed=11, p_rated=0.3)


def _sequential(spec):
    roster = make_roster(spec.roster_spec())
    rec = make_stream(spec.stream_spec(), spec.total_matches, spec.players, K=spec.team_size)
    res = BatchRater().rate(roster, rec, spec.team_size)
    return roster, res


def test_windows_equal_one_sequential_pass():
    summary, roster = run(SPEC, "cpu")
    ref, res = _sequential(SPEC)
    assert torch.equal(roster.state.nan_to_num(-7), ref.state.nan_to_num(-7))
    assert summary["matches"] == SPEC.total_matches and summary["windows"] == 5
    assert summary["rated"] == float((res.status == 0).sum())


def test_checkpoint_resume_after_injected_crash(tmp_path):
    d = str(tmp_path / "ck")
    with pytest.raises(InjectedFault):
        run(SPEC, "cpu", checkpoint_dir=d, checkpoint_every=1, fault_kill_after=2)
    saved, meta = checkpoint.load(os.path.join(d, "latest"))
    assert meta["windows_done"] == 2 and meta["next_offset"] == 600
    summary, roster = run(SPEC, "cpu", checkpoint_dir=d, checkpoint_every=1)
    assert summary["resumed_from_window"] == 2 and summary["matches"] == 1250 - 600
    ref, _ = _sequential(SPEC)
    assert torch.equal(roster.state.nan_to_num(-7), ref.state.nan_to_num(-7))  # exactly once
    # the re-rated windows reproduce the uninterrupted run's output records
    full, _ = run(SPEC, "cpu")
    assert sorted(summary["window_digests"]) == [2, 3, 4]
    for g in (2, 3, 4):
        assert summary["window_digests"][g] == full["window_digests"][g]


def test_output_records_accounted_for():
    """Every participant record of every window reaches the host sink, and the
    device digest counts the same records."""
    seen = []
    host, _ = run(SPEC, "cpu", records="host", on_records=lambda base, h: seen.append(
        (base, int(h["s_mu"].shape[0]), int((~torch.isnan(h["s_mu"])).sum()))))
    dig, _ = run(SPEC, "cpu")
    assert [b for b, _, _ in seen] == [0, 300, 600, 900, 1200]
    assert sum(m for _, m, _ in seen) == SPEC.total_matches
    assert host["participant_records"] == dig["participant_records"] == sum(p for _, _, p in seen)
    _, res = _sequential(SPEC)
    assert dig["participant_records"] == float((~torch.isnan(res.s_mu)).sum())
    assert dig["match_records"] == float(((res.status <= 2)).sum())


def test_checkpoint_falls_back_to_old_after_torn_replace(tmp_path):
    d = str(tmp_path / "ck")
    run(SPEC, "cpu", checkpoint_dir=d, checkpoint_every=2)
    latest = os.path.join(d, "latest")
    os.replace(latest, latest + ".old")  # crash between the two renames of a replace
    mgr = checkpoint.CheckpointManager(d)
    got = mgr.latest()
    assert got is not None and got[1]["windows_done"] == 4


def test_checkpoint_rejects_foreign_run(tmp_path):
    d = str(tmp_path / "ck")
    run(SPEC, "cpu", checkpoint_dir=d, checkpoint_every=2)
    other = RerateSpec(total_matches=1250, players=80, team_size=3, window=300, seed=12)
    with pytest.raises(ValueError):
        run(other, "cpu", checkpoint_dir=d)


def test_checkpoint_roundtrip_is_safetensors(tmp_path):
    roster = make_roster(SPEC.roster_spec())
    checkpoint.save(str(tmp_path / "c"), roster, {"x": 1})
    checkpoint.save(str(tmp_path / "c"), roster, {"x": 2})  # atomic replace
    r2, meta = checkpoint.load(str(tmp_path / "c"))
    assert meta["x"] == 2 and r2.epoch is None
    assert torch.equal(r2.state.nan_to_num(-7), roster.state.nan_to_num(-7))
    assert sorted(os.listdir(str(tmp_path))) == ["c"]


def _dp_rerate(rank, size, spec, sweeps):
    summary, roster = run(spec, "cpu", sweeps=sweeps)
    return {"state": roster.state, "summary": summary}


@pytest.mark.parametrize("sweeps", [1, 2])
def test_time_axis_sharded_rerate_two_ranks(tmp_path, sweeps):
    spec = RerateSpec(total_matches=1200, players=500, team_size=3, window=200, seed=5)
    res = run_ranks(_dp_rerate, 2, tmp_path, spec, sweeps)
    assert torch.equal(res[0]["state"].nan_to_num(-7), res[1]["state"].nan_to_num(-7))
    assert res[0]["summary"]["matches"] == 1200 and res[0]["summary"]["windows"] == 3
    ref, _ = _sequential(spec)
    mu, rmu = res[0]["state"][:, 0], ref.state[:, 0]
    ok = ~torch.isnan(rmu)
    assert torch.equal(ok, ~torch.isnan(mu))
    err = (mu[ok] - rmu[ok]).abs()
    if sweeps == 1:  # one merge: an approximation (parallel/accuracy.py quantifies it)
        assert float(err.median()) < 25.0
    else:  # sweeps == ranks: the exact sequential result up to fp32 rounding
        assert float(err.max()) < 0.05


def test_checkpoint_format3_and_older_formats(tmp_path):
    """Format 3 keeps the 7 tracks' (mu, sigma) (56 B per player: the spare granule is
    NULL in every row) + the attributes in their own file, no tags; format-1 (full
    [P, 32] rows) and format-2 (base rows + attrs) directories still load, tags reset."""
    from safetensors.torch import load_file, save_file
    import json

    roster = make_roster(SPEC.roster_spec())
    roster.state.view(-1, 8, 4)[:, :, 1::2] = 3.0  # tags: never saved
    checkpoint.save(str(tmp_path / "c3"), roster, {"x": 1})
    t = load_file(str(tmp_path / "c3" / checkpoint.TENSORS))
    assert sorted(t) == ["tracks"] and tuple(t["tracks"].shape) == (SPEC.players, 14)
    assert tuple(load_file(str(tmp_path / "c3" / checkpoint.ATTRS))["attrs"].shape) == (SPEC.players, 4)
    r3, meta = checkpoint.load(str(tmp_path / "c3"))
    assert meta["format"] == 3 and meta["spare_saved"] is False
    base = lambda s: s.view(-1, 8, 4)[:, :, 0::2].nan_to_num(-7)  # noqa: E731
    assert torch.equal(base(r3.state), base(roster.state))
    assert torch.equal(r3.attrs.nan_to_num(-7), roster.attrs.nan_to_num(-7))
    assert float(r3.state.view(-1, 8, 4)[:, :, 1::2].abs().max()) == 0.0
    # a non-NULL spare granule is kept
    odd = make_roster(SPEC.roster_spec())
    odd.state[0, 28] = 5.0
    checkpoint.save(str(tmp_path / "c3s"), odd, {})
    ro, mo = checkpoint.load(str(tmp_path / "c3s"))
    assert mo["spare_saved"] is True and float(ro.state[0, 28]) == 5.0
    for fmt, tensors in ((1, {"state": roster.state.contiguous(), "attrs": roster.attrs.contiguous()}),
                         (2, {"base": checkpoint.base_and_attrs(roster)[0].contiguous(),
                              "attrs": roster.attrs.contiguous()})):
        d = tmp_path / ("c%d" % fmt)
        d.mkdir()
        save_file(tensors, str(d / checkpoint.TENSORS))
        (d / checkpoint.META).write_text(json.dumps({"format": fmt, "windows_done": 3}))
        r, m = checkpoint.load(str(d))
        assert m["windows_done"] == 3 and torch.equal(base(r.state), base(roster.state))
        assert float(r.state.view(-1, 8, 4)[:, :, 1::2].abs().max()) == 0.0


def test_static_attrs_are_hard_linked(tmp_path):
    """A run whose attributes never change writes them once: the later checkpoints
    hard-link the previous file (no bytes written)."""
    roster = make_roster(SPEC.roster_spec())
    ck = checkpoint.AsyncCheckpointer("cpu", SPEC.players, fsync=False, static_attrs=True)
    p = str(tmp_path / "latest")
    for i in range(3):
        ck.submit(p, roster, {"windows_done": i + 1})
        ck.flush()
    assert os.stat(os.path.join(p, checkpoint.ATTRS)).st_nlink == 1  # the older dirs are gone
    assert ck.bytes == 3 * SPEC.players * 14 * 4 + SPEC.players * 4 * 4
    r, meta = checkpoint.load(p)
    assert meta["windows_done"] == 3 and torch.equal(r.attrs.nan_to_num(-7), roster.attrs.nan_to_num(-7))


def test_async_checkpointer_on_host(tmp_path):
    """The asynchronous writer's host path: two buffers, back-pressure, every
    submitted checkpoint committed by flush, the last one wins."""
    roster = make_roster(SPEC.roster_spec())
    ck = checkpoint.AsyncCheckpointer("cpu", SPEC.players, buffers=2, fsync=False)
    p = str(tmp_path / "latest")
    for i in range(5):
        roster.state[:, 0].add_(1.0)
        ck.submit(p, roster, {"windows_done": i + 1})
    ck.flush()
    assert ck.written == 5
    r, meta = checkpoint.load(p)
    assert meta["windows_done"] == 5
    assert torch.equal(r.state[:, 0].nan_to_num(-7), roster.state[:, 0].nan_to_num(-7))


def test_rerate_merge_precision_default():
    """BASELINE config 5 names fp16 moments: one-sweep re-rates merge in fp16 by default,
    causal re-sweeps in fp32 (their prefixes telescope)."""
    from analyzer_amd.runtime.rerate import default_comm_dtype

    assert default_comm_dtype(1) == "fp16" and default_comm_dtype(2) == "fp32"
