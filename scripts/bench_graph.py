#!/usr/bin/env python3
"""Streaming micro-batches against a device-resident roster: eager launches
(BatchRater.rate: schedule prepass + dataflow launch) vs one HIP graph replay
per batch (ops/graph.py GraphRater).  Each batch is synchronised, as a worker
committing batch by batch would."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.graph import GraphRater  # noqa: E402
from analyzer_amd.ops.rate import BatchRater  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=500)
    ap.add_argument("--batches", type=int, default=300)
    ap.add_argument("--team-size", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    K, B, N = args.team_size, args.batch, args.batches
    stream = make_stream(StreamSpec(team_size=K, seed=3), B * N, args.players, K=K, device=dev)
    res = {}
    for mode in ("eager", "graph", "eager", "graph"):
        roster = make_roster(RosterSpec(num_players=args.players, seed=2), device=dev)
        if mode == "graph":
            gr = GraphRater(roster, K, capacity=B)
            run = gr.rate
        else:
            br = BatchRater()
            run = lambda b, br=br, roster=roster: br.rate(roster, b, K, check=False)  # noqa: E731
        for i in range(10):  # warm-up
            run(stream[i * B:(i + 1) * B])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(N):
            run(stream[i * B:(i + 1) * B])
            torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / N
        res.setdefault(mode, []).append(us)
        print("%-5s %8.1f us/batch of %d  (%.3g matches/s)" % (mode, us, B, B / us * 1e6), flush=True)
    print(json.dumps({"batch": B, "players": args.players,
                      "us_per_batch": {k: min(v) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
