#!/usr/bin/env python3
"""One standalone K8 aggregation of a 10M-match 3v3 window (~400M events), for
rocprofv3 counter passes: python scripts/tele_once.py [--matches 1e7]."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.synth import StreamSpec, make_stream  # noqa: E402
from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, allocate_stats, make_telemetry  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--matches", type=float, default=1e7)
    ap.add_argument("--players", type=float, default=1e6)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M, P, K = int(args.matches), int(args.players), 3
    rec = make_stream(StreamSpec(team_size=K, seed=3), M, P, K=K, device=dev)
    tel = make_telemetry(TelemetrySpec(seed=4, min_events=20, max_events=60), rec, K)
    stats = allocate_stats(M, K, dev)
    for _ in range(args.reps):
        aggregate(tel, K, stats)
    torch.cuda.synchronize()
    print("events", tel.num_events)


if __name__ == "__main__":
    main()
