#!/usr/bin/env python3
"""Where does a co-running prepass hurt the executor?  Times, for n prepass CUs,
the dataflow launch and the schedule prepass alone and together, each on the
full chip or on HIP CU masks (n CUs for the prepass, the other 256 - n for the
executor with a 2 * (256 - n) workgroup grid):

    python scripts/cu_split.py --cus 32,64 --rounds 3

Rows: ``rate`` / ``sched`` alone on their masks, then both launched together
(``pair``), each one's span from its own events.  If the pair's rate span
exceeds the masked rate alone, the two interfere through the memory side (the
CUs are disjoint); if it does not, the pair is bound by the slower partner.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.native import native  # noqa: E402
from analyzer_amd.ops.rate import BatchRater, RateResult  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402


def span(stream, fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    with torch.cuda.stream(stream):
        fn()
    b.record(stream)
    return a, b


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--matches", type=int, default=10_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--cus", default="32,64")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P, M, K = args.players, args.matches, args.team_size
    recs = [make_stream(StreamSpec(team_size=K, seed=5 + i, p_afk=0.0), M, P, device=dev) for i in range(2)]
    roster = make_roster(RosterSpec(num_players=P, seed=1), device=dev)
    out = RateResult.allocate(M, K, dev)
    full = torch.cuda.current_stream(dev)
    rows = []
    for rnd in range(args.rounds):
        for n in [0] + [int(x) for x in args.cus.split(",")]:
            if n:
                es = torch.cuda.ExternalStream(native().cu_masked_stream(0, n, True), device=dev)
                ps = torch.cuda.ExternalStream(native().cu_masked_stream(0, n, False), device=dev)
                br = BatchRater(blocks=2 * (256 - n))
            else:
                es = ps = full
                br = BatchRater(blocks=512)
            res = {"round": rnd, "prepass_cus": n}
            # alone: the rating (on its mask), then the prepass (on its mask)
            sched = br.schedule(recs[0], K, P, tag="_a")
            torch.cuda.synchronize()
            a, b = span(es, lambda: br.rate(roster, recs[0], K, out=out, schedule=sched, check=False))
            torch.cuda.synchronize()
            res["rate_alone_ms"] = a.elapsed_time(b)
            a, b = span(ps, lambda: br.schedule(recs[1], K, P, tag="_b"))
            torch.cuda.synchronize()
            res["sched_alone_ms"] = a.elapsed_time(b)
            if n:
                # together: both launched back to back from the host, disjoint CUs
                sched = br.schedule(recs[0], K, P, tag="_a")
                torch.cuda.synchronize()
                a0, b0 = span(es, lambda: br.rate(roster, recs[0], K, out=out, schedule=sched, check=False))
                a1, b1 = span(ps, lambda: br.schedule(recs[1], K, P, tag="_b"))
                torch.cuda.synchronize()
                res["pair_rate_ms"] = a0.elapsed_time(b0)
                res["pair_sched_ms"] = a1.elapsed_time(b1)
                res["pair_total_ms"] = max(a0.elapsed_time(b0), a0.elapsed_time(b1))
            br.check_errors(dev)
            print(json.dumps(res), flush=True)
            rows.append(res)


if __name__ == "__main__":
    main()
