#!/usr/bin/env python3
"""Sweep-DP accuracy of the bench's N > 1 shape for several (ranks, merges per step) pairs
(parallel/accuracy.py: the N ranks simulated on one GPU, one sweep, after one warm window):
how many merges each N needs for Spearman(mu - sigma) >= 0.995 and a records median
|d mu| <= 8 (the per-participant outputs of the last window, what the reference writes per
match).  Defaults: config 2 (10M 3v3 matches per rank and step over 1M players, bf16);
``--config 3`` 12.5M 5v5, ``--config 5`` 16M 3v3 over 10M players with fp16 messages.

    python scripts/merges_vs_ranks.py --config 5 --pairs 8x1,8x2,8x4,8x8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.synth import RosterSpec  # noqa: E402
from analyzer_amd.parallel.accuracy import run  # noqa: E402

ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
ap.add_argument("--pairs", default="2x1,2x2,2x4,4x2,4x4,4x8,8x4,8x8", help="RANKSxMERGES,...")
ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5])
ap.add_argument("--correct", type=int, default=1, help="causal record correction (1) or not (0)")
args = ap.parse_args()
K = 5 if args.config == 3 else 3
P = 10_000_000 if args.config == 5 else 1_000_000
M = {2: 10_000_000, 3: 12_500_000, 5: 16_000_000}[args.config]   # matches per rank and step
dtype = "fp16" if args.config == 5 else "bf16"
pairs = [tuple(int(x) for x in p.split("x")) for p in args.pairs.split(",")]
for ranks, k in pairs:
    tab = run(ranks, P, M // k, k, [1], device="cuda", team_size=K, seed=1, comm_dtype=dtype,
              p_rated=RosterSpec().p_rated, warm_windows=1, correct=bool(args.correct))
    sw = tab["sweeps"]["1"]
    sh, rec = sw["tracks"]["shared"], sw.get("records_shared_mu", {})
    print(json.dumps({"config": args.config, "team_size": K, "players": P, "ranks": ranks, "merges_per_step": k,
                      "matches_per_rank_per_merge": M // k, "comm_dtype": dtype,
                      "dmu_median": sh["dmu_median"], "dmu_p99": sh["dmu_p99"],
                      "spearman_mu_minus_sigma": sh["spearman_mu_minus_sigma"],
                      "records_dmu_median": rec.get("dmu_median"), "records_dmu_p99": rec.get("dmu_p99"),
                      "records_dmu_max": rec.get("dmu_max"), "clamps": sw.get("clamp_hits")}), flush=True)
    torch.cuda.empty_cache()
