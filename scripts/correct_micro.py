"""The causal record correction on one device (round 5): the records pass of one
DP window (``native().correct_records``: 1.25M 3v3 matches over 1M players, the
k = 8 window of config 2) and the decode with / without the fused delta table,
alone on the GPU -- bench.py's merge_ms reports them beside the next prepass.

    python scripts/correct_micro.py [--matches 1.25e6] [--players 1e6]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from analyzer_amd.ops.native import native
from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from analyzer_amd.parallel.sweep import SweepMerger
from merge_micro import time_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=float, default=1e6)
    ap.add_argument("--matches", type=float, default=1.25e6)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    P, M, K = int(a.players), int(a.matches), 3
    roster = make_roster(RosterSpec(num_players=P, seed=3), device=dev)
    rec = make_stream(StreamSpec(team_size=K, seed=4), M, P, device=dev)
    m = SweepMerger(P, dev, comm_dtype="bf16", force=True)
    m.begin(roster)
    out = BatchRater().rate(roster, rec, K)
    m.messages_packed(roster)
    prefix = m.msg.clone()  # a non-zero prefix: this window's own messages
    delta = torch.empty((P, 16), device=dev)
    res = {"players": P, "matches": M}
    res["decode_ms"] = time_ms(lambda: m.decode_packed(roster, into=None), a.reps)
    res["decode_with_delta_ms"] = time_ms(lambda: m.decode_packed(roster, into=None, prefix=prefix, delta=delta),
                                          a.reps)
    res["correct_records_ms"] = time_ms(lambda: native().correct_records(rec, K, out.packed, delta), a.reps)
    # the same pass with no player in range (no delta reads): its row traffic alone
    res["correct_no_gather_ms"] = time_ms(lambda: native().correct_records(rec, K, out.packed, delta[:1]), a.reps)
    # a read + write of the rows at copy speed, for reference
    res["rows_rw_ms"] = time_ms(lambda: out.packed.mul_(1.0), a.reps)
    # the delta reads alone: the 2K players' 64-B lines of every match (a gather + sum)
    ids = rec[:, :2 * K].long().clamp_(0, P - 1)
    res["gather_only_ms"] = time_ms(lambda: delta.view(P, 8, 2)[:, :2].reshape(P, 4)[ids].sum(), a.reps)
    # traffic of the records pass: rows read + written, records, 2 x 2K 8-B gathers
    res["correct_GBps"] = (M * (2 * out.packed.shape[1] * 4 + (2 * K + 2) * 4) + M * 4 * K * 8) / 1e6 / \
        res["correct_records_ms"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
