#!/usr/bin/env python3
"""Fused vs separate telemetry aggregation across batch sizes (BASELINE config 4).

    python scripts/tele_batch.py [--sizes 500,2000,10000,100000,1000000,10000000]

For each batch of M 3v3 matches (20-60 events each) against a device-resident
1M-player roster, one batch is: schedule + rating launch, and either
  fused    -- the events folded by the rating launch itself (inline K8, one launch)
  separate -- the one-hot MFMA aggregation kernel after the rating launch
  rating   -- no telemetry (the floor)
  auto     -- the default: BatchRater.rate given the events picks fused up to
              ANA_TELE_FUSE_MAX matches, separate above
timed as the streaming worker sees it: host wall clock from the first enqueue
to the synchronize that ends the batch (median over reps, modes interleaved).
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.rate import BatchRater, RateResult  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402
from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, allocate_stats, make_telemetry  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes", default="500,2000,10000,100000,1000000,10000000")
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--events", default="20,60")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P, K = args.players, args.team_size
    lo, hi = (int(x) for x in args.events.split(","))
    roster = make_roster(RosterSpec(num_players=P, seed=1), device=dev)
    rater = BatchRater()
    forced = BatchRater()
    forced.tele_fuse_max = 1 << 62  # "fused": inline at every size
    for M in (int(x) for x in args.sizes.split(",")):
        reps = max(5, min(200, 2_000_000 // M))
        nb = 4  # distinct batches, cycled
        recs = [make_stream(StreamSpec(team_size=K, seed=11 + b), M, P, K=K, base=b * M, device=dev)
                for b in range(nb)]
        tspec = TelemetrySpec(seed=3, min_events=lo, max_events=hi)
        tele = [make_telemetry(tspec, recs[b], K, base=b * M) for b in range(nb)]
        stats = allocate_stats(M, K, dev)
        out = RateResult.allocate(M, K, dev)
        times = {"rating": [], "fused": [], "separate": [], "auto": []}
        for r in range(reps + 2):
            for mode in times:
                b = r % nb
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode in ("fused", "auto"):
                    t = tele[b]
                    (forced if mode == "fused" else rater).rate(roster, recs[b], K, out=out, check=False,
                                                                telemetry=(t.evoff, t.events, stats))
                else:
                    rater.rate(roster, recs[b], K, out=out, check=False)
                    if mode == "separate":
                        aggregate(tele[b], K, stats)
                torch.cuda.synchronize()
                if r >= 2:
                    times[mode].append((time.perf_counter() - t0) * 1e6)
        rater.check_errors(dev)
        row = {"matches": M, "events": int(sum(t.num_events for t in tele) / nb), "reps": reps}
        for mode, v in times.items():
            row[mode + "_us"] = round(statistics.median(v), 1)
        row["fused_vs_separate"] = round(row["fused_us"] / row["separate_us"], 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
