"""Time the K5 levelizers on one window: device dataflow (csrc/levels.hip) vs the
host walk.  python3 scripts/levels_time.py [--matches 1e7] [--players 1e6] [--team-size 3]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.native import native  # noqa: E402
from analyzer_amd.ops.rate import BatchRater  # noqa: E402
from analyzer_amd.ops.synth import StreamSpec, make_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matches", type=float, default=1e7)
    ap.add_argument("--players", type=float, default=1e6)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--skew", type=int, default=1)
    a = ap.parse_args()
    M, P, K = int(a.matches), int(a.players), a.team_size
    dev = torch.device("cuda:0")
    rec = make_stream(StreamSpec(team_size=K, seed=5, skew=a.skew), M, P, K=K, device=dev)
    br = BatchRater()
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = br.schedule(rec, K, P, tag="_lv")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ld, dd = native().levels_device(rec, K, P, s.link, s.deps)
        t2 = time.perf_counter()
        print("device: schedule %.2f ms + levels %.2f ms, depth %d" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, dd),
              flush=True)
    rh = rec.cpu()
    t0 = time.perf_counter()
    lh, dh = native().levels(rh, K, P)
    t1 = time.perf_counter()
    print("host walk: %.1f ms, depth %d, identical %s" % ((t1 - t0) * 1e3, dh, bool(torch.equal(ld.cpu(), lh))),
          flush=True)


if __name__ == "__main__":
    main()
