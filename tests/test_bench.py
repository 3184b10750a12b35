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
    # config 5 (10M players): one merge per step meets the fidelity bars at N = 8
    assert bench.parse(["--gpus", "8", "--config", "5"]).merges_per_step == 1
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


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_rank_json_contract_on_cpu(tmp_path, n):
    """The N > 1 path of the driver contract end to end on the CPU (``--device cpu``:
    host mirror, gloo): bench.py spawns its own N ranks (127.0.0.1 rendezvous), runs
    one-prepass-per-step DP steps with a merge after each of k = N windows, and rank 0
    prints ONE JSON line with the N > 1 keys -- the rank count, the merge split with the
    prepass placement, the accuracy block with the per-participant record errors and
    the merge decodes' clamp count."""
    import json
    import subprocess

    env = dict(os.environ, ANA_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    for var in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(var, None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--device", "cpu", "--gpus", str(n),
                          "--players", "2000", "--matches-per-gpu", str(1000 * n), "--steps", "2", "--warmup", "1"],
                         cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    j = json.loads(lines[0])
    k = min(n, 8)
    assert j["n_gpus"] == n and j["rccl_world"] == n and j["dist_backend"] == "gloo" and j["device"] == "cpu"
    # the mode names the backend that merged (a gloo rehearsal never claims RCCL)
    assert "gloo posterior merge" in j["config"]["mode"] and "RCCL" not in j["config"]["mode"]
    assert j["config"]["parallelism"] == "dp%d" % n and j["config"]["merges_per_step"] == k
    assert j["value"] == pytest.approx(n * 1000 * n / (j["ms_per_step"] / 1000.0))
    mm = j["merge_ms"]
    assert mm["prepass_placement"] and mm["buckets"] >= 1
    assert mm["collective"]  # which exchange merged (split / scan / bucketed all-reduce)
    acc = j["accuracy"]
    for key in ("records_dmu_median", "records_dmu_p99", "records_dmu_max", "spearman_mu_minus_sigma"):
        assert acc[key] is not None, key
    assert acc["merge_clamp_hits"] == 0
