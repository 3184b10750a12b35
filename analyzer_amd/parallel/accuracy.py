"""Accuracy of sweep data parallelism against the reference's exact semantics.

The reference rates every match in ``created_at`` order, one after another
(/root/reference/worker.py:176,191-192).  Sweep DP (parallel/sweep.py) lets N
ranks rate N consecutive time slices of a window at once and merges the
posteriors; ``sweeps`` causal re-sweeps shrink the error to fp32 rounding at
``sweeps == N``.  This module measures that error:

* ``simulate_sweep_dp`` runs N ranks **in one process** (one device) with the
  same kernels and the same stage order as the distributed merger -- messages,
  the exclusive prefix over ranks, the all-reduce -- summed in rank order.  It
  reproduces what RCCL computes up to the reduction order of fp32 sums, and it
  lets one GPU (or the CPU) measure 8-rank accuracy at full bench scale.
* ``exact`` rates the same time slices sequentially on one roster (the
  executor is exact per player, so this is the reference's result).
* ``compare`` reports, per track, the median / p99 / max of |d mu| over players,
  the sigma ratio, the Spearman correlation of the conservative skill mu - sigma,
  and the same |d mu| for the per-participant output records of the last window.

    python -m analyzer_amd.parallel.accuracy --ranks 8 --players 1e6 \\
        --matches-per-rank 1e7 --windows 1 --sweeps 1,2,4,8 [--device cuda]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..config import MODES
from ..ops.rate import BatchRater, RateResult, Roster
from ..ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from ..ops.native import native
from .sweep import COMM_DTYPES, SweepMerger

TRACKS = ["shared"] + list(MODES)


def _quantize(buf: torch.Tensor, comm_dtype: str) -> torch.Tensor:
    """What the collective carries: the 14 message columns in the comm dtype."""
    if comm_dtype == "fp32":
        return buf.clone()
    out = buf.clone()
    out[:, :14] = buf[:, :14].to(COMM_DTYPES[comm_dtype]).float()
    return out


def simulate_sweep_dp(rater: BatchRater, roster: Roster, shards: Sequence[torch.Tensor], K: int,
                      sweeps: int = 1, comm_dtype: str = "fp32",
                      outs: Optional[List[RateResult]] = None, correct: bool = True) -> List[RateResult]:
    """Rate one window split into ``len(shards)`` time slices the way N ranks of
    sweep DP would, updating ``roster`` to the merged result.  Returns the
    per-rank outputs of the last sweep; with ``correct`` (one sweep) each rank's
    records carry the causal record correction (the prefix of the earlier ranks'
    messages, in the wire dtype, summed in rank order)."""
    N = len(shards)
    mergers = [SweepMerger(roster.num_players, roster.device, rater.cfg, comm_dtype=comm_dtype,
                           sweeps=sweeps, world_size=N) for _ in range(N)]
    rosters = [roster.clone() for _ in range(N)]
    if outs is None:
        outs = [RateResult.allocate(int(s.shape[0]), K, roster.device) for s in shards]
    for m, ro in zip(mergers, rosters):
        m.begin(ro)
    for s in range(sweeps):
        for r in range(N):
            rater.rate(rosters[r], shards[r], K, out=outs[r])
            mergers[r].rated()
        msgs = []
        for m, ro in zip(mergers, rosters):
            m.messages(ro)
            msgs.append(_quantize(m.buf, comm_dtype))
        if s + 1 < sweeps:  # causal re-sweep: prior_r = start + messages of ranks < r
            acc = torch.zeros_like(msgs[0])
            for r in range(N):
                m = mergers[r]
                if m.prior is None:
                    m.prior = torch.empty_like(m.start)
                m.buf.copy_(acc)
                m.decode(rosters[r], into=m.prior)
                acc = acc + msgs[r]
        else:  # final merge: every rank decodes start + all messages
            total = torch.zeros_like(msgs[0])
            for r, x in enumerate(msgs):
                if correct and sweeps == 1:
                    # the causal record correction of rank r's records by the messages of
                    # the ranks before it, against the window start (parallel/sweep.py)
                    m = mergers[r]
                    if comm_dtype == "fp32":  # raw messages: the prefix is the increment table
                        delta = total
                    else:
                        delta = torch.empty((m.P, 16), dtype=torch.float32, device=roster.device)
                        native().prefix_delta(m.start, total[:, :14].to(COMM_DTYPES[comm_dtype]).contiguous(),
                                              rosters[r].attrs, m.vst, float(rater.cfg.unknown_player_sigma), delta)
                    native().correct_records(shards[r], K, outs[r].packed, delta.contiguous())
                total = total + x
            total = _quantize(total, comm_dtype)  # what the collective delivers: summed, rounded once
            for m, ro in zip(mergers, rosters):
                m.buf.copy_(total)
                m.decode(ro, into=m.start)
    roster.state.copy_(rosters[0].state)
    roster.epoch = rosters[0].epoch
    global CLAMPS
    CLAMPS += max(m.clamp_hits() for m in mergers)  # (the final decode is the same sum on every rank)
    return outs


CLAMPS = 0  # decodes held at the precision floor in the simulations since the last run()


def _spearman(a: torch.Tensor, b: torch.Tensor) -> float:
    if a.numel() < 2:
        return 1.0
    ra = torch.argsort(torch.argsort(a)).double()
    rb = torch.argsort(torch.argsort(b)).double()
    ra -= ra.mean()
    rb -= rb.mean()
    return float((ra * rb).sum() / (ra.norm() * rb.norm()).clamp_min(1e-30))


def _q(x: torch.Tensor, q: float) -> float:
    if x.numel() == 0:
        return 0.0
    x = x.double()
    if x.numel() > 1 << 24:  # quantile() caps its input size
        x = x[torch.randperm(x.numel(), device=x.device)[: 1 << 24]]
    return float(torch.quantile(x, q))


def compare(approx: Roster, exact: Roster, out_a: Optional[List[RateResult]] = None,
            out_e: Optional[List[RateResult]] = None) -> Dict[str, object]:
    """Error statistics of ``approx`` against ``exact`` (see the module doc)."""
    res: Dict[str, object] = {"tracks": {}}
    for t, name in enumerate(TRACKS):
        ma, sa = approx.state[:, 4 * t], approx.state[:, 4 * t + 2]
        me, se = exact.state[:, 4 * t], exact.state[:, 4 * t + 2]
        null_mismatch = int((torch.isnan(ma) != torch.isnan(me)).sum())
        ok = ~torch.isnan(ma) & ~torch.isnan(me)
        if int(ok.sum()) == 0:
            continue
        d = (ma[ok] - me[ok]).abs()
        ratio = sa[ok] / se[ok]
        res["tracks"][name] = {
            "players": int(ok.sum()), "null_mismatch": null_mismatch,
            "dmu_median": _q(d, 0.5), "dmu_p99": _q(d, 0.99), "dmu_max": float(d.max()),
            "sigma_ratio_median": _q(ratio, 0.5), "sigma_ratio_p01": _q(ratio, 0.01),
            "sigma_ratio_p99": _q(ratio, 0.99),
            "spearman_mu_minus_sigma": _spearman(ma[ok] - sa[ok], me[ok] - se[ok]),
        }
    if out_a is not None and out_e is not None:  # per-rank record lists, same slices
        ds = []
        n = 0
        for a, e in zip(out_a, out_e):
            ok = (a.status == 0) & (e.status == 0)
            d = (a.s_mu[ok] - e.s_mu[ok]).abs()
            ds.append(d[~torch.isnan(d)])
            n += int(ok.sum())
        d = torch.cat(ds)
        res["records_shared_mu"] = {"matches": n, "dmu_median": _q(d, 0.5),
                                    "dmu_p99": _q(d, 0.99), "dmu_max": float(d.max()) if d.numel() else 0.0}
    return res


def run(ranks: int, players: int, matches_per_rank: int, windows: int, sweeps: Sequence[int],
        device="cpu", team_size: int = 3, seed: int = 11, comm_dtype: str = "fp32",
        p_rated: float = 0.3, warm_windows: int = 0, correct: bool = True) -> Dict[str, object]:
    """Accuracy table: exact sequential vs sweep DP at each sweep count.
    ``warm_windows``: exact windows rated first (shared by both), so the
    comparison starts from a settled roster rather than fresh priors."""
    global CLAMPS
    dev = torch.device(device)
    K = team_size
    rater = BatchRater()
    base = make_roster(RosterSpec(num_players=players, seed=seed, p_rated=p_rated), device=dev)
    spec = StreamSpec(team_size=K, seed=seed + 1)
    M = matches_per_rank
    off = 0
    for _ in range(warm_windows):
        for r in range(ranks):  # slice by slice: a window of N slices may exceed one launch
            rater.rate(base, make_stream(spec, M, players, K=K, base=off, device=dev), K)
            off += M
    shard_sets = []
    for w in range(windows):
        shard_sets.append([make_stream(spec, M, players, K=K, base=off + (w * ranks + r) * M, device=dev)
                           for r in range(ranks)])
    t0 = time.perf_counter()
    exact = base.clone()
    out_e = None
    for shards in shard_sets:  # the global order: rank 0's slice, then rank 1's, ...
        out_e = [rater.rate(exact, sh, K) for sh in shards]
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    table = {"ranks": ranks, "players": players, "matches_per_rank": M, "windows": windows,
             "warm_windows": warm_windows, "team_size": K, "comm_dtype": comm_dtype,
             "device": str(dev), "exact_s": time.perf_counter() - t0, "sweeps": {},
             "records_corrected": bool(correct)}
    for S in sweeps:
        t0 = time.perf_counter()
        approx = base.clone()
        outs = None
        CLAMPS = 0
        for shards in shard_sets:
            outs = simulate_sweep_dp(rater, approx, shards, K, sweeps=S, comm_dtype=comm_dtype, correct=correct)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        stats = compare(approx, exact, outs, out_e)
        stats["clamp_hits"] = CLAMPS  # decodes held at the precision floor (0 = none)
        stats["elapsed_s"] = time.perf_counter() - t0
        table["sweeps"][str(S)] = stats
    return table


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--players", type=float, default=20000)
    ap.add_argument("--matches-per-rank", type=float, default=200000)
    ap.add_argument("--windows", type=int, default=2)
    ap.add_argument("--warm-windows", type=int, default=1)
    ap.add_argument("--sweeps", default="1,2,4")
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--comm-dtype", default="fp32", choices=sorted(COMM_DTYPES))
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--no-correct", action="store_true",
                    help="records without the causal record correction (parallel/sweep.py)")
    args = ap.parse_args(argv)
    sweeps = [int(x) for x in args.sweeps.split(",") if x]
    table = run(args.ranks, int(args.players), int(args.matches_per_rank), args.windows, sweeps,
                device=args.device, team_size=args.team_size, seed=args.seed,
                comm_dtype=args.comm_dtype, warm_windows=args.warm_windows, correct=not args.no_correct)
    print(json.dumps(table, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
