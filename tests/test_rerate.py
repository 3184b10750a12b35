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


def _dp_rerate(rank, size, spec):
    summary, roster = run(spec, "cpu")
    return {"state": roster.state, "summary": summary}


def test_time_axis_sharded_rerate_two_ranks(tmp_path):
    spec = RerateSpec(total_matches=1200, players=500, team_size=3, window=200, seed=5)
    res = run_ranks(_dp_rerate, 2, tmp_path, spec)
    assert torch.equal(res[0]["state"].nan_to_num(-7), res[1]["state"].nan_to_num(-7))
    assert res[0]["summary"]["matches"] == 1200 and res[0]["summary"]["windows"] == 3
    # sweep merge stays close to the exact sequential result on a sparse history
    ref, _ = _sequential(spec)
    mu, rmu = res[0]["state"][:, 0], ref.state[:, 0]
    ok = ~torch.isnan(rmu)
    assert torch.equal(ok, ~torch.isnan(mu))
    assert float((mu[ok] - rmu[ok]).abs().median()) < 25.0
