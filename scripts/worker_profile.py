#!/usr/bin/env python3
"""Per-stage profile of the streaming worker (where do the ~2.6 ms
of a 500-match batch go when the GPU work is ~47 us?).

    python scripts/worker_profile.py --synthetic 100000 [--store columnar://] [--engine native]

Runs worker.py's synthetic path in-process with ANA_TRACE=1 and reports, per
stage (utils/trace.py ranges: load, rate.rows, rate.encode_h2d, rate.launch,
rate.d2h, rate.finish, commit, ack), the total and per-batch milliseconds, the broker
delivery overhead (everything else inside the consuming loop), the end-to-end
matches/s, and the top functions by own time (cProfile) -- one JSON object.
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--synthetic", type=int, default=100000)
    ap.add_argument("--store", default="columnar://")
    ap.add_argument("--engine", default="native")
    ap.add_argument("--batchsize", type=int, default=500)
    ap.add_argument("--cprofile", type=int, default=1)
    ap.add_argument("--pipeline", default="false", help="PIPELINE: two batches in flight (true) or one")
    ap.add_argument("--segments", type=int, default=1, help="time the stream in this many parts")
    args = ap.parse_args()
    os.environ["ANA_TRACE"] = "1"
    os.environ["DATABASE_URI"] = args.store
    os.environ["ENGINE"] = args.engine
    os.environ["BATCHSIZE"] = str(args.batchsize)
    os.environ["PIPELINE"] = args.pipeline
    os.environ.setdefault("IDLE_TIMEOUT", "0.01")
    import logging

    from analyzer_amd.config import WorkerConfig
    from analyzer_amd.runtime import broker as B
    from analyzer_amd.runtime.source import populate, publish
    from analyzer_amd.runtime.worker import Worker
    from analyzer_amd.utils import trace

    logging.getLogger("__name__").setLevel(logging.WARNING)
    w = Worker(WorkerConfig.from_env(), broker=B.MemoryBroker()).connect()
    matches = populate(w.store, args.synthetic, 2 * args.synthetic, team_size=3, seed=1)
    ids = [m if isinstance(m, str) else m.api_id for m in matches]
    # warm up (graph capture, first-touch of the roster) on the first batch, untimed
    publish(w.channel, w.cfg.queue, ids[:args.batchsize])
    w.start_consuming()
    trace.clear()
    rest = ids[args.batchsize:]
    seg = -(-len(rest) // args.segments)
    n0 = w.stats.matches
    pr = cProfile.Profile() if args.cprofile else None
    dt, rates = 0.0, []
    for k in range(0, len(rest), seg):  # segments: the box's host is shared, report the spread
        publish(w.channel, w.cfg.queue, rest[k:k + seg])
        m0 = w.stats.matches
        t0 = time.perf_counter()
        if pr:
            pr.enable()
        w.start_consuming()
        if pr:
            pr.disable()
        d = time.perf_counter() - t0
        dt += d
        rates.append((w.stats.matches - m0) / d)
    n = w.stats.matches - n0
    rates.sort()
    batches = max(1, (n + args.batchsize - 1) // args.batchsize)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for e in trace.events():
        tot[e["name"]] += e["dur"] / 1000.0
        cnt[e["name"]] += 1
    stages = {k: {"ms_total": round(v, 2), "ms_per_batch": round(v / batches, 4), "calls": cnt[k]}
              for k, v in sorted(tot.items(), key=lambda kv: -kv[1])}
    top = []
    if pr:
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        top = [ln for ln in s.getvalue().splitlines() if ln.strip()][:40]
    print(json.dumps({"matches": n, "seconds": round(dt, 3), "matches_per_s": round(n / dt),
                      "segments": len(rates), "segment_matches_per_s_median": round(rates[len(rates) // 2]),
                      "segment_matches_per_s_min": round(rates[0]), "segment_matches_per_s_max": round(rates[-1]),
                      "ms_per_batch": round(dt * 1000.0 / batches, 4), "batchsize": args.batchsize,
                      "store": args.store, "engine": args.engine, "cprofile": bool(pr),
                      "pipeline": bool(w._pipe),
                      "stages": stages}, indent=1))
    for ln in top:
        print(ln)


if __name__ == "__main__":
    main()
