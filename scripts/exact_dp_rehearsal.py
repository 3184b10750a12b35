"""Exact DP (C2, parallel/exact_dp.py) rehearsal on one device: N gloo ranks
share the GPU, rate one window round by round, and report rounds, collectives
and wall time per window next to one device rating it alone.

    python scripts/exact_dp_rehearsal.py --ranks 2 --matches 1000000 --players 100000
"""
import argparse
import json
import os
import sys
import os
import socket
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, size, port, a, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    from analyzer_amd.ops.rate import BatchRater
    from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
    from analyzer_amd.parallel.exact_dp import RoundPlan, rate_exact_dp, rounds

    dev = torch.device("cuda:0")
    rec = make_stream(StreamSpec(team_size=a.team_size, seed=5), a.matches, a.players, K=a.team_size, device=dev)
    level, depth = rounds(rec, a.team_size, a.players)
    times = []
    for it in range(a.repeats + 1):
        roster = make_roster(RosterSpec(num_players=a.players, seed=4), device=dev)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rate_exact_dp(BatchRater(), roster, rec, a.team_size, level=level)
        torch.cuda.synchronize()
        dist.barrier()
        if it:  # the first window warms up allocations and the gloo buffers
            times.append(time.perf_counter() - t0)
    if rank == 0:
        plan = RoundPlan(level, size)
        roster = make_roster(RosterSpec(num_players=a.players, seed=4), device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        BatchRater().rate(roster, rec, a.team_size)
        torch.cuda.synchronize()
        single = time.perf_counter() - t0
        q.put({"ranks": size, "matches": a.matches, "players": a.players, "team_size": a.team_size,
               "rounds": plan.n_rounds, "collectives_per_window": plan.n_rounds, "max_slice": plan.max_slice,
               "exact_dp_window_s": min(times), "single_device_window_s": single,
               "backend": "gloo (host-staged, all ranks on one GPU)"})
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--matches", type=int, default=1000000)
    ap.add_argument("--players", type=int, default=100000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=2)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_rank, args=(a.ranks, _port(), a, q), nprocs=a.ranks, join=True)
    print(json.dumps(q.get()))


if __name__ == "__main__":
    main()
