#!/usr/bin/env python3
"""Time the schedule prepass and the dataflow launch separately, A/B-ing
executor knobs interleaved in one process (guide §5.4 rule 24).

    python scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 \\
        --local 0,1 --diag 1

patterns: random (uniform players, or ``--skew`` power law), serial (every
match has the same 2K players: chain depth = M, the pure hop latency), disjoint
(no player repeats: nothing ever waits).  ``--diag 1`` runs the timing build
(ANA_RATE_DIAG) and prints the per-iteration wait/iteration clocks.
"""
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
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--matches", type=int, default=10_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--blocks", default="512")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--idle", default="8", help="ANA_RATE_IDLE values (max idle sleep rounds)")
    ap.add_argument("--tight", default="-1", help="ANA_RATE_TIGHT values (2K lanes per match; -1 auto)")
    ap.add_argument("--local", default="1", help="ANA_RATE_LOCAL values (LDS local hand-off; 1 = the default)")
    ap.add_argument("--diag", default="0", help="ANA_RATE_DIAG values (timing build)")
    ap.add_argument("--skew", type=int, default=1)
    ap.add_argument("--rated", type=float, default=1.0,
                    help="fraction of players with stored ratings (1.0 = steady state, no seeding)")
    ap.add_argument("--pattern", default="random", choices=["random", "serial", "disjoint"])
    ap.add_argument("--touch", default="0",
                    help="1: read the whole roster after the prepass, untimed, so the launch starts with "
                         "its rows warm in the Infinity Cache; 2: the same with the native warm_rows "
                         "kernel inside the timed launch (ANA_ROSTER_WARM); comma list to A/B")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P, M, K = args.players, args.matches, args.team_size
    rec = make_stream(StreamSpec(team_size=K, seed=5, p_afk=0.0, skew=args.skew), M, P, device=dev)
    if args.pattern == "serial":      # every match has the same 2K players: chain depth = M
        rec[:, :2 * K] = torch.arange(2 * K, dtype=torch.int32, device=dev)
    elif args.pattern == "disjoint":  # no player repeats: nothing ever waits
        assert P >= 2 * K * M, "disjoint pattern needs players >= 2K * matches"
        rec[:, :2 * K] = (torch.arange(M, dtype=torch.int32, device=dev)[:, None] * (2 * K)
                          + torch.arange(2 * K, dtype=torch.int32, device=dev)[None, :])
    out = RateResult.allocate(M, K, dev)
    results = {}
    sink = torch.zeros(256, dtype=torch.int32, device=dev)  # --touch 2 scratch
    combos = [(int(b), int(i), int(t), int(lo), int(d), int(sp)) for b in args.blocks.split(",")
              for i in args.idle.split(",") for t in args.tight.split(",")
              for lo in args.local.split(",") for d in args.diag.split(",") for sp in args.touch.split(",")]
    for rnd in range(args.rounds):
        for b, idle, tg, loc, dg, sp in combos:
            os.environ["ANA_RATE_TIGHT"] = str(tg)
            os.environ["ANA_RATE_IDLE"] = str(idle)
            os.environ["ANA_RATE_LOCAL"] = str(loc)
            os.environ["ANA_RATE_DIAG"] = str(dg)
            key = "b%d/i%d/t%d/local%d/diag%d" % (b, idle, tg, loc, dg) + ("/touch%d" % sp if sp else "")
            roster = make_roster(RosterSpec(num_players=P, seed=1, p_rated=args.rated,
                                            p_mode_rated=args.rated), device=dev)
            br = BatchRater(blocks=b)
            br.schedule(rec, K, P)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sched = br.schedule(rec, K, P)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if sp == 2:  # the engine's warm-up kernel, timed with the launch
                from analyzer_amd.ops.native import native

                native().warm_rows(roster.state, sink)
            elif sp:  # roster rows warm in the Infinity Cache (untimed)
                float(roster.state.sum())
                torch.cuda.synchronize()
                t0 += time.perf_counter() - t1
                t1 = time.perf_counter()
            br.rate(roster, rec, K, out=out, schedule=sched, check=False)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            br.check_errors(dev)
            stale = br.stale_retries(dev)
            d = br.diag(dev)
            results.setdefault(key, []).append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, d))
            line = ("round %d %s schedule %7.2f ms rate %8.2f ms stale %d iterations %d (%.2f matches/it)"
                    " hand-offs local %d global %d" % (rnd, key, (t1 - t0) * 1e3, (t2 - t1) * 1e3, stale,
                                                       d["wave_iterations"], M / max(d["wave_iterations"], 1),
                                                       d["local_handoffs"], d["global_handoffs"]))
            if dg:
                line += " | worked iterations %d (%.2f matches each): issue %.3f + wait %.3f + after %.3f us" % (
                    d["worked_iterations"], d["matches_per_worked_iteration"], d["issue_us"], d["wait_us"],
                    d["after_us"])
                line += " [prior %.3f update %.3f publish %.3f rest %.3f]" % (
                    d["after_prior_us"], d["after_update_us"], d["after_publish_us"], d["after_rest_us"])
                line += " issue [ready %.3f assign %.3f loads %.3f polls %.3f]" % (
                    d["issue_ready_us"], d["issue_assign_us"], d["issue_loads_us"], d["issue_polls_us"])
                line += " near-ready %.2f of %.1f pending" % (d["near_ready_per_worked_iteration"],
                                                               d["pending_per_worked_iteration"])
            if args.pattern == "serial":
                line += " | %.3f us per hop" % ((t2 - t1) * 1e6 / M)
            print(line, flush=True)
    summary = {k: {"schedule_ms_min": min(x[0] for x in v), "rate_ms_min": min(x[1] for x in v),
                   "rate_ms_median": sorted(x[1] for x in v)[len(v) // 2], "diag_last": v[-1][2]}
               for k, v in results.items()}
    print(json.dumps({"pattern": args.pattern, "players": P, "matches": M, "team_size": K,
                      "skew": args.skew, "by_config": summary}))


if __name__ == "__main__":
    main()
