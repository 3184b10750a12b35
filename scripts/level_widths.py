#!/usr/bin/env python3
"""Dependency-level width profile of a synthetic window (host levelizer, CPU).

    python scripts/level_widths.py --matches 1e7 --players 1e6 --team-size 3

Prints the DAG depth, the level by which given fractions of the matches are
done, and how many levels fall below given widths.  A window whose levels are
all about equally wide has no thin tail for a following window to fill.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from analyzer_amd.ops.native import native  # noqa: E402
from analyzer_amd.ops.synth import StreamSpec, make_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--matches", type=float, default=1e7)
    ap.add_argument("--players", type=float, default=1e6)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--skew", type=int, default=1)
    ap.add_argument("--seed", type=int, default=2025)
    args = ap.parse_args()
    M, P, K = int(args.matches), int(args.players), args.team_size
    rec = make_stream(StreamSpec(team_size=K, seed=args.seed, skew=args.skew), M, P, K=K)
    lv, depth = native().levels(rec, K, P)
    lv = lv.numpy()
    w = np.bincount(lv[lv > 0])[1:]
    cum = np.cumsum(w) / w.sum()
    done = {str(f): int(np.searchsorted(cum, f)) + 1 for f in (0.5, 0.7, 0.8, 0.9, 0.95, 0.99)}
    below = {str(t): [int((w < t).sum()), float(w[w < t].sum() / w.sum())] for t in (16000, 8000, 4000, 1000)}
    print(json.dumps({"matches": M, "players": P, "team_size": K, "skew": args.skew, "depth": int(depth),
                      "mean_width": float(w.mean()), "width_at": {str(i): int(w[i - 1]) for i in (1, 10, 100, 300, 500, 700, 800) if i <= len(w)},
                      "level_by_fraction_done": done, "levels_below_width_and_their_match_share": below}))


if __name__ == "__main__":
    main()
