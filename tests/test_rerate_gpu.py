"""Re-rate device paths (``-m gpu``): the fused window digest (csrc/digest.hip) against
the fp64 torch digest of the same rows, its run-to-run determinism, and the
asynchronous checkpoint writer (runtime/checkpoint.py) on device rosters."""
import os

import numpy as np
import pytest
import torch

from analyzer_amd.ops import rate as R
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from analyzer_amd.runtime import checkpoint
from analyzer_amd.runtime.rerate import _Digest, window_digest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,M,P", [(3, 200_000, 20_000), (5, 50_000, 5_000), (1, 3_000, 400), (3, 1, 10)])
def test_device_digest_matches_fp64_torch(gpu_device, K, M, P):
    roster = make_roster(RosterSpec(num_players=P, seed=3, p_rated=0.4), device=gpu_device)
    rec = make_stream(StreamSpec(team_size=K, seed=4, p_afk=0.05), M, P, K=K, device=gpu_device)
    res = R.BatchRater().rate(roster, rec, K)
    torch.cuda.synchronize()
    dig = _Digest()
    hist = torch.full((256,), 5, dtype=torch.int64, device=gpu_device)
    a = dig(res, K, hist)
    b = dig(res, K)
    ref = window_digest(res)
    assert a.shape == ref.shape
    assert torch.equal(a, b)  # deterministic: fixed grid, fixed-order sums
    # the status counts are added to the histogram: every match once
    want = torch.bincount(res.status.to(torch.int64), minlength=256) + 5
    assert torch.equal(hist, want)
    a, ref = a.cpu().numpy(), ref.cpu().numpy()
    assert a[0] == ref[0] and a[1] == ref[1]  # counts are exact
    np.testing.assert_allclose(a[2:], ref[2:], rtol=1e-12, atol=1e-6)


def test_async_checkpoint_roundtrip_on_device(gpu_device, tmp_path):
    roster = make_roster(RosterSpec(num_players=100_000, seed=9, p_rated=0.5), device=gpu_device)
    mgr = checkpoint.CheckpointManager(str(tmp_path / "ck"), every=1)
    assert mgr.maybe_save(1, roster, {"x": 1})
    before = roster.state.clone()
    roster.state[:, 0].add_(1.0)  # the rating goes on while the writer runs
    assert mgr.maybe_save(2, roster, {"x": 2})
    roster.state[:, 0].add_(1.0)
    mgr.flush()
    got, meta = mgr.latest(gpu_device)
    assert meta["windows_done"] == 2 and meta["format"] == checkpoint.FORMAT
    want = before.clone()
    want[:, 0].add_(1.0)
    base = lambda s: s.view(-1, 8, 4)[:, :, 0::2].nan_to_num(-7)  # noqa: E731
    assert torch.equal(base(got.state), base(want))
    assert torch.equal(got.attrs.nan_to_num(-7), roster.attrs.nan_to_num(-7))
    assert float(got.state.view(-1, 8, 4)[:, :, 1::2].abs().max()) == 0.0  # tags are not saved


def test_prepared_checkpoint_buffers(gpu_device, tmp_path):
    """CheckpointManager.prepare allocates the pinned buffers (and the static attributes'
    host copy) before the first save; the saves then write what a lazily prepared writer
    writes."""
    roster = make_roster(RosterSpec(num_players=50_000, seed=19, p_rated=0.5), device=gpu_device)
    out = {}
    for tag, prep in (("lazy", False), ("prepared", True)):
        mgr = checkpoint.CheckpointManager(str(tmp_path / tag), every=1, static_attrs=True)
        if prep:
            mgr.prepare(roster)
            assert mgr._async is not None and mgr._async._host
        assert mgr.maybe_save(1, roster, {"x": 1})
        mgr.flush()
        assert mgr.stats()["checkpoints"] == 1.0
        out[tag] = mgr.latest(gpu_device)[0]
    a, b = out["lazy"], out["prepared"]
    assert torch.equal(a.state.nan_to_num(-7), b.state.nan_to_num(-7))
    assert torch.equal(a.attrs.nan_to_num(-7), b.attrs.nan_to_num(-7))
