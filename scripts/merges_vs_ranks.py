#!/usr/bin/env python3
"""Sweep-DP accuracy of the bench's N > 1 shape (10M 3v3 / 12.5M 5v5 matches per rank and step,
1M players, bf16 messages, one sweep, after one warm window) for several
(ranks, merges per step) pairs: how many merges each N needs for Spearman(mu - sigma)
>= 0.99 and a records median |d mu| <= 15 (the per-participant outputs of the last
window, what the reference writes per match; parallel/accuracy.py, the N ranks
simulated on one GPU)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.synth import RosterSpec  # noqa: E402
from analyzer_amd.parallel.accuracy import run  # noqa: E402

pairs = [tuple(int(x) for x in p.split("x")) for p in (sys.argv[1] if len(sys.argv) > 1 else
                                                      "2x1,2x2,2x4,4x2,4x4,4x8,8x4,8x8").split(",")]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3          # team size (5: bench config 3)
M = 10_000_000 if K == 3 else 12_500_000                  # matches per rank and step
for ranks, k in pairs:
    tab = run(ranks, 1_000_000, M // k, k, [1], device="cuda", team_size=K, seed=1, comm_dtype="bf16",
              p_rated=RosterSpec().p_rated, warm_windows=1)
    sw = tab["sweeps"]["1"]
    sh, rec = sw["tracks"]["shared"], sw.get("records_shared_mu", {})
    print(json.dumps({"team_size": K, "ranks": ranks, "merges_per_step": k, "matches_per_rank_per_merge": M // k,
                      "dmu_median": sh["dmu_median"], "dmu_p99": sh["dmu_p99"],
                      "spearman_mu_minus_sigma": sh["spearman_mu_minus_sigma"],
                      "records_dmu_median": rec.get("dmu_median"), "records_dmu_p99": rec.get("dmu_p99"),
                      "records_dmu_max": rec.get("dmu_max")}), flush=True)
    torch.cuda.empty_cache()
