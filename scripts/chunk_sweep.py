#!/usr/bin/env python3
"""Executor time of one window vs matches per ticket (chunk_len 16/32/64): fewer
matches held per wave for short DP windows.  python scripts/chunk_sweep.py [M]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.rate import BatchRater, RateResult  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402


class Fixed(BatchRater):
    def __init__(self, cl):
        super().__init__()
        self.cl = cl

    def chunk_len(self, M, telemetry=False):
        return self.cl


M = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000
dev = torch.device("cuda:0")
K, P = 3, 1_000_000
rec = make_stream(StreamSpec(team_size=K, seed=5, p_afk=0.0), M, P, device=dev)
out = RateResult.allocate(M, K, dev)
roster = make_roster(RosterSpec(num_players=P, seed=1), device=dev)
for rnd in range(3):
    for cl in (64, 32, 16):
        br = Fixed(cl)
        sched = br.schedule(rec, K, P)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        br.rate(roster, rec, K, out=out, schedule=sched, check=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        br.check_errors(dev)
        print("round %d matches %d chunk_len %d rate %.3f ms" % (rnd, M, cl, dt), flush=True)
