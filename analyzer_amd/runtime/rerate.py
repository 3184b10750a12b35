"""Full-history re-rate driver (SURVEY P4 + C5 + C4; BASELINE configs 3 and 5).

The reference is online-only: batches of <= 500 matches in arrival order, no
way to re-rate a history (/root/reference/worker.py:18,176).  This driver
streams a long synthetic history through the engine window by window:

* the history is a counter-RNG stream, so window ``g`` of rank ``r`` is
  generated on the device from its global offset -- no host I/O, and any window
  can be regenerated after a crash;
* one rank: windows are rated exactly, in order (dataflow engine, prepass of
  window g+1 overlapped with rating g -- runtime/engine.py);
* N ranks (one per GPU): time-axis sharding -- global window g is N
  consecutive blocks of ``window`` matches, rank r rates block r exactly from
  the window-start roster, then one RCCL all-reduce of natural-parameter
  messages merges the blocks (sweep mode, parallel/sweep.py);
* every ``checkpoint_every`` windows the replicated roster and the stream
  position are checkpointed atomically; a restarted run resumes from there and
  produces the same roster as an uninterrupted run (exactly-once);
* every window's per-participant output records (the reference writes them per
  match, /root/reference/rater.py:151-169, committed per batch at
  worker.py:194) are accounted for: ``records="digest"`` reduces them on the
  device to a count + fp64 column sums per window (a resumed run reproduces the
  digests of the windows it re-rates); ``records="host"`` streams them D2H into
  a ring of pinned buffers on a copy stream, overlapped with the next windows
  (double-buffered device outputs), and hands them to ``on_records``;
* status counters are accumulated on the device and reduced over ranks (C4);
  the executor's error flags are sticky over windows and checked before every
  checkpoint, so a failed middle window is never checkpointed over.

    python -m analyzer_amd.runtime.rerate --matches 1000000000 --players 10000000 \\
        --window 16000000 --team-size 3 --checkpoint-dir /tmp/ck
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import deque
from dataclasses import asdict, dataclass
from typing import Callable, Dict, Optional

import torch

from ..config import EngineConfig, RaterConfig
from ..ops import rate as R
from ..ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from ..parallel.comm import broadcast_roster, init_from_env, reduce_counts, world
from ..parallel.sweep import SweepMerger
from ..utils.trace import trace_range
from .checkpoint import CheckpointManager
from .engine import WindowPipeline
from .ingest import OutputSink


class InjectedFault(SystemExit):
    """Raised by ``fault_kill_after`` to simulate a crash (exit code 17)."""


@dataclass
class RerateSpec:
    total_matches: int
    players: int
    team_size: int = 3
    window: int = 1_000_000          # matches per rank per window
    seed: int = 2024
    p_afk: float = 0.02
    p_rated: float = 0.0             # fraction of players with a stored rating at start

    def roster_spec(self) -> RosterSpec:
        return RosterSpec(num_players=self.players, seed=self.seed, p_rated=self.p_rated)

    def stream_spec(self) -> StreamSpec:
        return StreamSpec(team_size=self.team_size, seed=self.seed + 1, p_afk=self.p_afk)


def default_comm_dtype(sweeps: int) -> str:
    """Merge message precision when none is given: fp16 for one sweep -- BASELINE config 5
    names fp16 moments, and bench.py --config 5 merges in fp16 (8 ranks x 16M matches over
    10M players: roster Spearman 0.9988, 0 clamps, profiles/r6/fidelity_config5.log) --
    and fp32 for causal re-sweeps, whose prefixes must telescope exactly."""
    return "fp16" if int(sweeps) <= 1 else "fp32"


def n_windows(spec: RerateSpec, size: int) -> int:
    per = spec.window * size
    return (spec.total_matches + per - 1) // per


def window_slice(spec: RerateSpec, g: int, rank: int, size: int):
    """[lo, hi) global match offsets of rank's block of window g."""
    lo = g * spec.window * size + rank * spec.window
    hi = min(lo + spec.window, spec.total_matches)
    return lo, max(lo, hi)


class _Digest:
    """Per-window digests on the device: one deterministic streaming pass over the
    packed output rows (csrc/digest.hip) -- 7 torch nansum passes and a bincount
    before, 8.5 ms per 16M-match window (profiles/r6/rerate_attribution.log).  With
    ``hist`` (int64[256] on the rows' device) the pass also adds the window's status
    counts to it, in place of a strided copy + bincount of the status bytes (the host
    path counts with a bincount)."""

    def __init__(self):
        self._scratch = {}

    def device(self, res: R.RateResult) -> bool:
        return res.packed is not None and res.packed.is_cuda

    def __call__(self, res: R.RateResult, K: int, hist: Optional[torch.Tensor] = None) -> torch.Tensor:
        rows = res.packed
        if not self.device(res):
            if hist is not None:
                hist += torch.bincount(res.status.to(torch.int64), minlength=256)
            return window_digest(res)
        from ..ops.native import native

        key = (rows.device, K)
        if key not in self._scratch:
            self._scratch[key] = torch.empty(native().records_digest_scratch(K), dtype=torch.float64,
                                             device=rows.device)
        out = torch.empty(3 + 10 * K, dtype=torch.float64, device=rows.device)
        native().records_digest(rows, K, self._scratch[key], out, hist)
        return out


def window_digest(res: R.RateResult) -> torch.Tensor:
    """[2 + 5*2K + 1] fp64: matches with records (rated / AFK / invalid),
    participant records written (non-NULL shared mu), then the column sums of the
    five per-slot outputs and quality over written values (the host / unpacked
    path; on the device ``_Digest`` computes the same in one kernel)."""
    S = res.s_mu.shape[1]
    st = res.status
    wrote = (st == R.RATED) | (st == R.AFK) | (st == R.INVALID_ROSTERS)
    parts = [wrote.sum().to(torch.float64).view(1),
             (~torch.isnan(res.s_mu)).sum().to(torch.float64).view(1)]
    for t in (res.s_mu, res.s_sig, res.delta, res.m_mu, res.m_sig):
        parts.append(torch.nansum(t, dim=0, dtype=torch.float64).view(S))
    parts.append(torch.nansum(res.quality, dtype=torch.float64).view(1))
    return torch.cat(parts)


def run(spec: RerateSpec, device=None, checkpoint_dir: Optional[str] = None,
        checkpoint_every: int = 1, fault_kill_after: Optional[int] = None,
        on_window: Optional[Callable[[int, R.RateResult], None]] = None,
        rater: Optional[R.BatchRater] = None, comm_dtype: Optional[str] = None,
        records: str = "digest", on_records: Optional[Callable[[int, dict], None]] = None,
        sweeps: int = 1):
    """Rate the whole history; returns (metrics reduced over ranks, final roster).

    ``records``: "digest" (device reduction per window, in the metrics as
    ``window_digests``), "host" (pinned D2H ring; ``on_records(base, host_dict)``
    gets every window's rows) or "none"."""
    if records not in ("digest", "host", "none"):
        raise ValueError("records must be digest, host or none")
    rank, size = world()
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    rater = rater or R.BatchRater(RaterConfig())
    K = spec.team_size
    # the rating kernels only read the attributes (csrc/dataflow.hip): written with the
    # first checkpoint, hard-linked into the later ones (runtime/checkpoint.py)
    ck = CheckpointManager(checkpoint_dir, checkpoint_every, rank=0, static_attrs=True)
    start_window = 0
    restored = ck.latest(dev)
    if restored is not None:
        roster, meta = restored
        if meta.get("spec") != asdict(spec) or meta.get("world") != size:
            raise ValueError("checkpoint in %s belongs to a different run" % checkpoint_dir)
        start_window = int(meta["windows_done"])
    else:
        roster = make_roster(spec.roster_spec(), device=dev)
        broadcast_roster(roster)  # C3 (identical by construction; keeps replicas honest)
    comm_dtype = comm_dtype or default_comm_dtype(sweeps)
    merger = (SweepMerger(spec.players, dev, rater.cfg, comm_dtype=comm_dtype, sweeps=sweeps)
              if size > 1 else None)
    pipe = WindowPipeline(rater, roster, K, merger=merger)
    total = n_windows(spec, size)
    counts = torch.zeros(256, dtype=torch.int64, device=dev)
    digests = {}
    digest = _Digest()
    sspec = spec.stream_spec()
    outs = [None, None]  # double-buffered: the sink copies one while the next is rated
    host_stats = {"windows": 0, "participant_records": 0}

    def took(base, host):
        host_stats["windows"] += 1
        host_stats["participant_records"] += int((~torch.isnan(host["s_mu"])).sum())
        if on_records is not None:
            on_records(base, host)

    sink = OutputSink(dev, took) if records == "host" else None
    if dev.type == "cuda":
        rater.clear_sticky(dev)

    def window_rec(g):
        lo, hi = window_slice(spec, g, rank, size)
        return make_stream(sspec, hi - lo, spec.players, K=K, base=lo, device=dev)

    # ANA_RERATE_GEN=tail (default): the next window's records are generated in the rating's
    # tail on the prepass stream (needs the tail-overlapped prepass, no DP merge); main: on
    # the main stream between the ratings
    gen_tail = (os.environ.get("ANA_RERATE_GEN", "tail") == "tail" and dev.type == "cuda" and merger is None
                and pipe.side is not None and pipe.side != torch.cuda.current_stream(dev) and pipe.tail > 0)
    # the checkpoint writer's pinned buffers are set up before the run, like the roster
    # (ANA_CKPT_PREPARE=0: at the first save)
    if rank == 0 and os.environ.get("ANA_CKPT_PREPARE", "1") not in ("", "0", "false"):
        ck.prepare(roster)
    t0 = time.perf_counter()
    rated = 0
    D = pipe.depth  # windows prepared ahead (runtime/engine.py)
    ahead = deque(pipe.prepare(window_rec(j)) for j in range(start_window, min(start_window + D, total)))
    for g in range(start_window, total):
        cur = ahead.popleft()
        M = cur.rec.shape[0]
        b = g & 1
        if outs[b] is None or outs[b].quality.shape[0] != M:
            outs[b] = R.RateResult.allocate(M, K, dev)
        elif sink is not None and sink.copied(outs[b]) is not None:
            torch.cuda.current_stream(dev).wait_event(sink.copied(outs[b]))
        nw = g + D  # the window prepared behind this rating
        if gen_tail and nw < total:
            # window g+D is generated on the prepass stream in rate(g)'s tail, right before
            # its prepass, instead of on the main stream in front of rate(g)
            res = pipe.rate(cur, out=outs[b])
            side = pipe.side
            with torch.cuda.stream(side):
                pipe.wait_tail(side)
                rec_next = window_rec(nw)
                made = torch.cuda.Event()
                made.record(side)
            rec_next.record_stream(torch.cuda.current_stream(dev))
            ahead.append(pipe.prepare(rec_next, produced=made))
        else:
            # window g+D is generated before rate(g) is enqueued; its prepass waits for the tail
            res, nxt = pipe.step(cur, window_rec(nw) if nw < total else None, out=outs[b])
            if nxt is not None:
                ahead.append(nxt)
        pipe.results_ready(res)  # the DP merge's deferred record correction of these rows
        if records == "digest":
            digests[g] = digest(res, K, counts)  # + the status counts
        else:
            counts += torch.bincount(res.status.to(torch.int64), minlength=256)
        if sink is not None:
            sink.push(window_slice(spec, g, rank, size)[0], res)
        rated += M
        if on_window is not None:
            on_window(g, res)
        if ck.due(g + 1):
            if dev.type == "cuda":  # never checkpoint over a failed window
                rater.check_errors(dev, sticky=True)
            if merger is not None:  # ... nor over a clamped merge decode
                merger.check()
            if rank == 0:
                with trace_range("checkpoint", window=g + 1):
                    ck.maybe_save(g + 1, roster, {"spec": asdict(spec), "world": size,
                                                  "next_offset": window_slice(spec, g + 1, 0, size)[0]})
        if fault_kill_after is not None and g + 1 >= fault_kill_after:
            # the simulated crash hits once the checkpoints submitted so far are
            # committed (asynchronous writes, runtime/checkpoint.py): a real crash
            # loses the ones still in flight and resumes from the one before
            ck.flush()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            raise InjectedFault(17)
    if sink is not None:
        sink.flush()
    ck.flush()  # the run ends when its last checkpoint is committed
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dev.type == "cuda":
        rater.check_errors(dev, sticky=True)
    if merger is not None:
        merger.check()
    c = counts.cpu()
    local = {R.STATUS_NAMES.get(i, str(i)): float(c[i]) for i in range(256) if int(c[i])}
    local["matches"] = float(rated)
    if records == "digest" and digests:
        d = torch.stack([digests[g] for g in sorted(digests)]).cpu()
        local["match_records"] = float(d[:, 0].sum())
        local["participant_records"] = float(d[:, 1].sum())
    elif records == "host":
        local["participant_records"] = float(host_stats["participant_records"])
        local["egress_bytes"] = float(sink.bytes)
    summed = reduce_counts(local, dev)
    summed["seconds"] = reduce_counts({"seconds": dt}, dev, op="max")["seconds"]
    summed["windows"] = float(total - start_window)
    summed["resumed_from_window"] = float(start_window)
    summed["matches_per_s"] = summed["matches"] / summed["seconds"] if summed["seconds"] > 0 else 0.0
    if rank == 0:
        summed.update({"checkpoint_" + k: v for k, v in ck.stats().items()})
    if records == "digest":
        summed["window_digests"] = {g: digests[g].cpu().tolist() for g in sorted(digests)}
    return summed, roster


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--matches", type=float, required=True)
    ap.add_argument("--players", type=float, required=True)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--window", type=float, default=1e6)
    ap.add_argument("--seed", type=int, default=2024)
    ecfg = EngineConfig.from_env()
    ap.add_argument("--checkpoint-dir", default=ecfg.checkpoint_dir)
    ap.add_argument("--checkpoint-every", type=int, default=ecfg.checkpoint_every)
    ap.add_argument("--fault-kill-after", type=int, default=None,
                    help="fault injection: exit(17) after this many windows")
    ap.add_argument("--device", default=None)
    ap.add_argument("--comm-dtype", default=ecfg.comm_dtype or None,
                    choices=["fp32", "fp16", "bf16"], help="sweep-merge message precision")
    ap.add_argument("--records", default="digest", choices=["digest", "host", "none"],
                    help="output records: device digest per window, pinned D2H stream, or dropped")
    ap.add_argument("--sweeps", type=int, default=ecfg.sweeps, help="causal sweeps per window (N ranks)")
    ap.add_argument("--digests", action="store_true", help="print every window's digest")
    args = ap.parse_args(argv)
    rank, size, dev = init_from_env()
    spec = RerateSpec(total_matches=int(args.matches), players=int(args.players),
                      team_size=args.team_size, window=int(args.window), seed=args.seed)
    try:
        res, roster = run(spec, args.device or dev, args.checkpoint_dir, args.checkpoint_every,
                          args.fault_kill_after, comm_dtype=args.comm_dtype, records=args.records,
                          sweeps=args.sweeps)
    except InjectedFault:
        if rank == 0:
            print(json.dumps({"fault_injected_after_windows": args.fault_kill_after}), flush=True)
        raise
    if rank == 0:
        digs = res.pop("window_digests", None)
        if digs is not None and not args.digests:  # a compact fingerprint instead of every window
            res["digest_fingerprint"] = float(sum(sum(v) for v in digs.values()))
        elif digs is not None:
            res["window_digests"] = digs
        import hashlib  # bit-exact: sha256 of every (mu, sigma) of the final roster

        res["roster_sha256"] = hashlib.sha256(
            roster.state[:, 0::2].contiguous().cpu().numpy().tobytes()).hexdigest()
        print(json.dumps(dict(res, n_ranks=size, spec=asdict(spec))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
