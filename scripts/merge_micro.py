"""Sweep-DP merge kernels on one device: the message kernel
(posterior vs prior -> natural-parameter messages) and the decode kernel
(start + summed messages -> roster and next start) at P = 1M and 10M players,
without the collective (bench.py --gpus N reports that part as merge_ms).

    python scripts/merge_micro.py --players 1e6,1e7
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from analyzer_amd.ops.synth import RosterSpec, make_roster
from analyzer_amd.parallel.sweep import SweepMerger


def time_ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", default="1e6,1e7")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = []
    for P in [int(float(x)) for x in a.players.split(",")]:
        roster = make_roster(RosterSpec(num_players=P, seed=3), device=dev)
        for dtype in ("fp32", "bf16"):
            m = SweepMerger(P, dev, comm_dtype=dtype, world_size=2)
            m.begin(roster)
            # a posterior that moved every rated row a little
            roster.state.view(P, 8, 4)[..., 0].add_(0.5)
            msg = time_ms(lambda: m.messages(roster), a.reps)
            dec = time_ms(lambda: m.decode(roster, into=m.start), a.reps)
            state_mb = P * 128 / 1e6
            extra = {}
            if dtype != "fp32":
                # what merge() runs for a compressed dtype: the fp32 path needs a split
                # into the comm operands and a join back; the packed kernels neither
                split = time_ms(lambda: m._join(m.buf, m._split(m.buf)), a.reps)
                extra = {"fp32_path_split_join_ms": split,
                         "packed_messages_ms": time_ms(lambda: m.messages_packed(roster), a.reps),
                         "packed_decode_ms": time_ms(lambda: m.decode_packed(roster, into=m.start), a.reps)}
                extra["packed_total_ms"] = extra["packed_messages_ms"] + extra["packed_decode_ms"]
                extra["fp32_path_total_ms"] = msg + dec + split
            out.append({"players": P, "comm_dtype": dtype, "messages_ms": msg, "decode_ms": dec, **extra,
                        "message_bytes_per_rank": m.comm_bytes,
                        # messages: read start + prior(=start) + roster + attrs, write buf
                        "messages_GBps": (3 * state_mb + P * 16 / 1e6 + P * 64 / 1e6) / msg,
                        "decode_GBps": (state_mb + P * 64 / 1e6 + P * 16 / 1e6 + 2 * state_mb) / dec})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
