#!/usr/bin/env python3
"""Time the schedule prepass and the dataflow launch separately for several
persistent-grid sizes, interleaved in one process (guide §5.4 rule 24)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.rate import BatchRater, RateResult  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--matches", type=int, default=10_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--blocks", default="128,256,512,1024,2048")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--idle", default="8", help="ANA_RATE_IDLE values (max idle sleep rounds)")
    ap.add_argument("--debug", default="0", help="ANA_RATE_DEBUG values (experiments)")
    ap.add_argument("--spec", default="0", help="ANA_RATE_SPEC values (speculative matches/iteration)")
    ap.add_argument("--tight", default="-1", help="ANA_RATE_TIGHT values (2K lanes per match; -1 auto)")
    ap.add_argument("--variant", default="0", help="ANA_RATE_VARIANT values (executor A/B variants)")
    ap.add_argument("--packed", default="1", help="output layout: 1 packed rows, 0 separate arrays")
    ap.add_argument("--hot", type=float, default=0.0)
    ap.add_argument("--rated", type=float, default=1.0,
                    help="fraction of players with stored ratings (1.0 = steady state, no seeding)")
    ap.add_argument("--pattern", default="random", choices=["random", "serial", "disjoint"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P, M, K = args.players, args.matches, args.team_size
    rec = make_stream(StreamSpec(team_size=K, seed=5, p_hot=args.hot, p_afk=0.0), M, P, device=dev)
    if args.pattern == "serial":      # every match has the same 2K players: chain depth = M
        rec[:, :2 * K] = torch.arange(2 * K, dtype=torch.int32, device=dev)
    elif args.pattern == "disjoint":  # no player repeats: nothing ever waits
        assert P >= 2 * K * M, "disjoint pattern needs players >= 2K * matches"
        rec[:, :2 * K] = (torch.arange(M, dtype=torch.int32, device=dev)[:, None] * (2 * K)
                          + torch.arange(2 * K, dtype=torch.int32, device=dev)[None, :])
    outs = {1: RateResult.allocate(M, K, dev), 0: RateResult.allocate(M, K, dev, packed=False)}
    results = {}
    for rnd in range(args.rounds):
        for b, idle, dbg, sp, tg, pk, va in [(int(x), int(y), int(z), int(w), int(v), int(u), int(t))
                                             for x in args.blocks.split(",") for y in args.idle.split(",")
                                             for z in args.debug.split(",") for w in args.spec.split(",")
                                             for v in args.tight.split(",") for u in args.packed.split(",")
                                             for t in args.variant.split(",")]:
            out = outs[pk]
            os.environ["ANA_RATE_TIGHT"] = str(tg)
            os.environ["ANA_RATE_IDLE"] = str(idle)
            os.environ["ANA_RATE_DEBUG"] = str(dbg)
            os.environ["ANA_RATE_SPEC"] = str(sp)
            os.environ["ANA_RATE_VARIANT"] = str(va)
            key = "b%d/i%d/d%d/s%d/t%d/p%d/v%d" % (b, idle, dbg, sp, tg, pk, va)
            roster = make_roster(RosterSpec(num_players=P, seed=1, p_rated=args.rated,
                                            p_mode_rated=args.rated), device=dev)
            br = BatchRater(blocks=b)
            br.schedule(rec, K, P)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sched = br.schedule(rec, K, P)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            br.rate(roster, rec, K, out=out, schedule=sched, check=False)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            br.check_errors(dev)
            stale = br.stale_retries(dev)
            iters = br.iterations(dev)
            results.setdefault(key, []).append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
            print("round %d %s schedule %7.2f ms rate %8.2f ms stale retries %d iterations %d "
                  "(%.2f matches/iteration)" % (rnd, key, (t1 - t0) * 1e3, (t2 - t1) * 1e3, stale,
                                                iters, M / max(iters, 1)), flush=True)
    summary = {b: {"schedule_ms_min": min(x[0] for x in v), "rate_ms_min": min(x[1] for x in v),
                   "rate_ms_median": sorted(x[1] for x in v)[len(v) // 2]} for b, v in results.items()}
    print(json.dumps({"pattern": args.pattern, "players": P, "matches": M, "team_size": K, "hot": args.hot,
                      "by_blocks": summary}))


if __name__ == "__main__":
    main()
