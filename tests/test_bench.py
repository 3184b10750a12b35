"""bench.py argument contract (CPU): BASELINE config defaults, the merge precision
default and the rank-count check that runs before any GPU call."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


@pytest.fixture(autouse=True)
def _clean_env(monkeypatch):
    for var in ("COMM_DTYPE", "SWEEPS", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(var, raising=False)


def test_config_defaults():
    a = bench.parse([])
    assert (a.config, a.team_size, a.matches_per_gpu, a.players) == (2, 3, 10_000_000, 1_000_000)
    a = bench.parse(["--config", "3"])
    assert (a.team_size, a.matches_per_gpu) == (5, 12_500_000)
    a = bench.parse(["--config", "5"])
    assert (a.players, a.matches_per_gpu, a.ring) == (10_000_000, 16_000_000, 2)
    a = bench.parse(["--config", "2", "--matches-per-gpu", "1250000"])
    assert a.matches_per_gpu == 1_250_000


def test_merge_precision_default(monkeypatch):
    # one sweep: bf16 messages (accuracy identical to fp32, profiles/r2/slice_size_accuracy.log;
    # fp32 range in RCCL's sums); config 5 keeps BASELINE's fp16 moments
    assert bench.parse([]).comm_dtype == "bf16"
    assert bench.parse(["--config", "5"]).comm_dtype == "fp16"
    # causal re-sweeps aim at the exact result: fp32 unless asked otherwise
    assert bench.parse(["--sweeps", "4"]).comm_dtype == "fp32"
    assert bench.parse(["--sweeps", "4", "--comm-dtype", "bf16"]).comm_dtype == "bf16"
    monkeypatch.setenv("COMM_DTYPE", "fp32")
    assert bench.parse([]).comm_dtype == "fp32"


def test_world_size_must_match_gpus(monkeypatch):
    # under torchrun, --gpus must equal WORLD_SIZE; checked before the GPU is touched
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="--gpus 3 but WORLD_SIZE=2"):
        bench.main(["--gpus", "3"])


def test_merges_per_step():
    a = bench.parse(["--merges-per-step", "8"])
    assert a.merges_per_step == 8 and a.matches_per_gpu == 10_000_000  # same matches per step
    with pytest.raises(SystemExit):
        bench.parse(["--merges-per-step", "3"])   # must divide the step
    with pytest.raises(SystemExit):
        bench.parse(["--config", "4", "--merges-per-step", "2"])


def test_merges_per_step_default_is_accuracy_bounded(monkeypatch):
    """One GPU has nothing to merge (one window per step); N > 1 merges N times per
    step so that one sweep keeps Spearman(mu - sigma) >= 0.99 against the exact
    sequential result (profiles/r3/merges_vs_ranks.log); causal re-sweeps are
    exact already and keep one window."""
    assert bench.parse([]).merges_per_step == 1
    # one merge per rank's worth of concurrency: k = the largest power of two <= N (<= 8)
    assert bench.parse(["--gpus", "8"]).merges_per_step == 8
    assert bench.parse(["--gpus", "4"]).merges_per_step == 4
    assert bench.parse(["--gpus", "6"]).merges_per_step == 4
    assert bench.parse(["--gpus", "2", "--config", "3"]).merges_per_step == 2
    # 5v5 has 10 appearances a match: twice the merges from N = 4 (merges_vs_ranks_5v5.log)
    assert bench.parse(["--gpus", "4", "--config", "3"]).merges_per_step == 8
    assert bench.parse(["--gpus", "8", "--config", "3"]).merges_per_step == 16
    assert bench.parse(["--gpus", "8", "--sweeps", "8"]).merges_per_step == 1
    assert bench.parse(["--gpus", "8", "--config", "4"]).merges_per_step == 1
    assert bench.parse(["--gpus", "8", "--merges-per-step", "2"]).merges_per_step == 2
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.parse([]).merges_per_step == 4
    assert bench.parse([]).accuracy == 1


def test_shared_card_blocks():
    """Ranks sharing a card (gloo rehearsal) split the executor grid; one rank per GPU
    (RCCL, or world <= GPUs) keeps the default."""
    assert bench.shared_card_blocks(8, 8, "nccl") == 0
    assert bench.shared_card_blocks(8, 1, "nccl") == 0
    assert bench.shared_card_blocks(2, 2, "gloo") == 0
    assert bench.shared_card_blocks(2, 1, "gloo") == 256
    assert bench.shared_card_blocks(8, 1, "gloo") == 64
    assert bench.shared_card_blocks(6, 2, "gloo") == 170
    assert bench.shared_card_blocks(64, 1, "gloo") == 16
