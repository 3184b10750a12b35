#!/usr/bin/env python3
"""Headline benchmark: matches/sec rated (whole node), 3v3 TrueSkill, 1M-player roster.

Metric/config from BASELINE.json.  One step = every rank rates its own window of
``--matches-per-gpu`` synthetic 3v3 matches (10M by default, BASELINE config 2)
against the replicated 1M-player roster, in exact per-player chronological
order (schedule prepass + one dataflow launch, both tracks, full output
records), then -- for N > 1 -- merges the per-player posteriors of all ranks
with an RCCL all-reduce of natural-parameter deltas (sweep DP, BASELINE
config 3 / north star).  Weak scaling: per-GPU work is fixed as N grows.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver launches N>1)

``python bench.py --gpus N`` (N > 1) without a torchrun environment starts its
own N ranks: child processes, one per GPU, before this process touches the
GPU; rank 0 prints the JSON line and the exit status is the worst child's.
``ANA_DIST_BACKEND=gloo`` rehearses N ranks on fewer GPUs (ranks share
devices; the merge goes through the host).

Synthetic data: roster and streams come from the on-device counter RNG
(random-init ratings), generated before the timed region like a prefetched
data loader; the timed region contains all rating work of every step.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

from analyzer_amd.config import EngineConfig

# reference rate: ~354 3v3 matches/s per CPU core for rater.rate_match
# (measured); the whole-node bound is 8 cores x 354 = 2832/s.
BASELINE_MATCHES_PER_S = 2832.0
# 5v5 (config 3): ~264 matches/s per core x 8 cores
BASELINE_5V5_MATCHES_PER_S = 2112.0


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (default: WORLD_SIZE, else 1); N > 1 without torchrun spawns N ranks")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the C++ host mirror on the CPU, ranks over gloo -- a rehearsal of this "
                         "driver contract (spawn, rendezvous, merges, the JSON line) without a GPU, for "
                         "tiny sizes only (tests/test_bench.py); every number it prints is a CPU number")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--matches-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--ring", type=int, default=4, help="distinct pre-generated windows per rank")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--check", action="store_true", help="also validate statuses after timing")
    ap.add_argument("--verify", action="store_true",
                    help="after timing, rate window 0 again on the device and on the fp64 host "
                         "mirror and report the deviations (ops/verify.py) in the JSON line")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5],
                    help="BASELINE config: 2 = 10M 3v3/GPU (headline), 3 = 12.5M 5v5/GPU (100M at DP=8), "
                         "4 = streaming: rating + per-event telemetry aggregation, "
                         "5 = full-history re-rate windows: 16M 3v3/GPU over a 10M-player roster, "
                         "fp16 merge messages")
    ap.add_argument("--skew", type=int, default=1,
                    help="player activity: floor(u^skew * P); 1 = uniform (headline), 2 = quadratic, "
                         "3 = cubic (SURVEY H1: ~585k dependency levels per 10M window)")
    ap.add_argument("--events", default="20,60", help="config 4: min,max telemetry events per match")
    ap.add_argument("--telemetry-mode", default="auto", choices=["auto", "overlap", "fused", "separate", "tail"],
                    help="config 4: auto = the rating launch takes the telemetry and fuses it up to "
                         "ANA_TELE_FUSE_MAX matches (worker batches; scripts/tele_batch.py), above that "
                         "(10M windows) the MFMA kernel as in tail, from 0.4; fused = always inline in the rating "
                         "groups; separate = the MFMA kernel after the rating on the same stream; "
                         "overlap = the MFMA kernel co-runs with the rating on its own stream; "
                         "tail = the MFMA kernel of window i starts on its own stream once the rating of "
                         "window i has claimed ANA_TELE_TAIL_AT (default 0.9) of its chunks, beside its "
                         "drain and the next prepass, and the next rating waits for it")
    ap.add_argument("--comm-dtype", default=None, choices=["fp32", "fp16", "bf16"],
                    help="sweep-merge message precision (N > 1; default COMM_DTYPE, else bf16 for one "
                         "sweep -- at 8 x 10M the compressed messages leave the sweep error unchanged, "
                         "profiles/r2/slice_size_accuracy.log, and RCCL's bf16 sums keep fp32's range "
                         "where fp16 sums of 8 ranks' mean shifts could overflow -- fp16 for config 5 "
                         "(BASELINE: fp16 moments) and fp32 for causal re-sweeps)")
    ap.add_argument("--merges-per-step", type=int, default=None,
                    help="N > 1: split each GPU's step into this many windows with a sweep merge after "
                         "each (same matches per step; shorter slices cut the sweep-DP error ~linearly, "
                         "profiles/r2/slice_size_accuracy.log).  Default: 1 on one GPU (nothing to "
                         "merge), N for N > 1 (largest power of two <= N, at most 8): every rank then "
                         "misses about the same (N - 1) / N of a step of the others' matches between merges, "
                         "and one sweep keeps Spearman(mu - sigma) >= 0.99 against the exact sequential "
                         "result -- 0.9993 / 0.9978 / 0.9948 at N = 2 / 4 / 8 for 10M 3v3 per rank over 1M "
                         "players (profiles/r3/merges_vs_ranks.log); 5v5 (config 3) doubles k from N = 4: "
                         "0.9897 at N = k = 4 but 0.9971 at k = 8, 0.9884 at N = k = 8 but 0.9965 at k = 16 "
                         "(profiles/r3/merges_vs_ranks_5v5.log)")
    ap.add_argument("--accuracy", type=int, default=1,
                    help="N > 1: after timing, rank 0 measures the sweep-DP error of this run's "
                         "configuration against the exact sequential rating (parallel/accuracy.py, "
                         "N ranks simulated on its GPU) and reports it in the JSON line (0 = skip)")
    ap.add_argument("--emulate-allreduce", default=None, metavar="N:GBps[:us]",
                    help="with --force-merge on one GPU: replace the (identity) all-reduce of every merge "
                         "by a stand-in that takes the modelled time of an N-rank ring all-reduce of the "
                         "operands at GBps bus bandwidth (+ us latency, default 25) and streams the buffer "
                         "on 16 CUs as RCCL's channels do -- a one-GPU projection of the N-GPU step "
                         "(parallel/sweep.py emulate); the prepass placement follows the modelled time")
    ap.add_argument("--force-merge", action="store_true",
                    help="N = 1: run the merge kernels after every window anyway (messages + decode, "
                         "no collective) -- prices the DP merge's device work against --merges-per-step")
    ap.add_argument("--sweeps", type=int, default=EngineConfig.from_env().sweeps,
                    help="causal sweeps per window (N > 1): 1 = one merge (approximate); "
                         "N = exact sequential semantics (parallel/sweep.py)")
    args = ap.parse_args(argv)
    if args.config == 3:
        args.team_size = 5
        if args.matches_per_gpu == 10_000_000:
            args.matches_per_gpu = 12_500_000
    if args.config == 4:
        args.ring = min(args.ring, 2)
    if args.config == 5:
        if args.players == 1_000_000:
            args.players = 10_000_000
        if args.matches_per_gpu == 10_000_000:
            args.matches_per_gpu = 16_000_000
        args.ring = min(args.ring, 2)
    if args.merges_per_step is None:
        n = args.gpus if args.gpus is not None else int(os.environ.get("WORLD_SIZE") or 1)
        k = 1
        while k * 2 <= min(n, 8):
            k *= 2
        if args.team_size == 5 and n >= 4:
            k *= 2      # 5v5: 10 appearances a match, twice the merges for the same error
        if args.config == 5:
            # 16M matches per rank over 10M players: ~1.2 appearances per player per rank and
            # window at k = 8, ~10 at k = 1 -- against 7.5 / 60 for config 2 -- so ONE merge per
            # step meets both fidelity bars at N = 8 (roster Spearman 0.9988 >= 0.995, records
            # median 3.45 <= 8, 0 clamps; profiles/r6/fidelity_config5.log) and the 320-MB
            # merge runs once per step instead of k times
            k = 1
        # k = 8 at N = 8 is the smallest k that meets both fidelity bars with the causal
        # record correction (simulated N = 8: records median 8.0 <= 15, roster Spearman
        # 0.9956 >= 0.995; k = 4 gives records 14.1 but roster Spearman 0.983 --
        # profiles/r5/record_correction.log)
        args.merges_per_step = k if n > 1 and args.config != 4 and args.sweeps <= 1 else 1
    if args.merges_per_step < 1 or args.matches_per_gpu % args.merges_per_step:
        ap.error("--merges-per-step must divide --matches-per-gpu")
    if args.merges_per_step > 1 and args.config == 4:
        ap.error("--merges-per-step is for the rating configs (2, 3, 5)")
    if args.comm_dtype is None:
        one_sweep = "fp16" if args.config == 5 else "bf16"
        args.comm_dtype = os.environ.get("COMM_DTYPE") or (
            "fp32" if args.sweeps > 1 else one_sweep)
    return args


def shared_card_blocks(world: int, ngpu: int, backend: str) -> int:
    """Executor grid for ranks that share a card (gloo rehearsals with more ranks than
    GPUs): each rank's persistent grid is sized to its share of the 512 blocks, so every
    rank's launch is resident at once -- full grids from 4-8 processes get time-sliced
    and trip the executor's 5-s no-progress watchdog
    (profiles/r3/dp_gloo_rehearsals_k_default.log).  0 = one rank per GPU (the default
    grid)."""
    if backend == "nccl" or not ngpu or world <= ngpu:
        return 0
    return max(16, 512 // -(-world // ngpu))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """Start ``n`` ranks of this benchmark as child processes (torchrun's
    environment contract, rendezvous on 127.0.0.1).  Nothing here touches the
    GPU: each child initialises its own device.  Returns the worst exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        failed = [c for c in codes if c not in (None, 0)]
        if failed:  # one rank died: the others would hang in a collective
            time.sleep(5)
            for i, p in enumerate(procs):
                if p.poll() is None:
                    p.kill()
                codes[i] = p.wait()
            break
        time.sleep(0.2)
    bad = [c for c in codes if c != 0]
    if bad:
        print("bench: rank exit codes %s" % codes, file=sys.stderr)
        return max(abs(c) for c in bad) or 1
    return 0


def main(argv=None) -> int:
    raw = list(sys.argv[1:] if argv is None else argv)
    args = parse(raw)
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or 1)
    if args.gpus > 1 and env_world is None:
        return spawn_ranks(args.gpus, raw)
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # one rank per GPU; ANA_DIST_BACKEND=gloo lets several ranks share one GPU to
    # rehearse the multi-process path on a 1-GPU box (production: nccl = RCCL)
    backend = EngineConfig.from_env().dist_backend
    cpu = args.device == "cpu"
    if cpu:
        backend = "gloo"
        dev = torch.device("cpu")
    else:
        ngpu = torch.cuda.device_count()
        local = local % ngpu if backend != "nccl" and ngpu else local
        blocks = shared_card_blocks(world, ngpu, backend)
        if blocks and not os.environ.get("ANA_RATE_BLOCKS"):
            os.environ["ANA_RATE_BLOCKS"] = str(blocks)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    from analyzer_amd.ops.rate import BatchRater, RateResult, NOT_PROCESSED
    from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
    from analyzer_amd.parallel.sweep import SweepMerger
    from analyzer_amd.runtime.engine import WindowPipeline

    P, M, K = args.players, args.matches_per_gpu, args.team_size
    sub = args.merges_per_step           # windows per step (a merge after each when N > 1)
    Mw = M // sub                        # matches per window and GPU
    roster = make_roster(RosterSpec(num_players=P, seed=args.seed), device=dev)
    spec = StreamSpec(team_size=K, seed=args.seed + 1, skew=args.skew)
    n_windows = max(1, min(args.ring, (args.steps + args.warmup) * sub))
    total_windows = (args.steps + args.warmup) * sub
    windows = [make_stream(spec, Mw, P, K=K, base=(w * world + rank) * Mw, device=dev)
               for w in range(n_windows)]
    rater = BatchRater()
    if args.telemetry_mode == "fused":
        rater.tele_fuse_max = 1 << 62  # inline at any launch size
    out = RateResult.allocate(Mw, K, dev)
    tele = stats = None
    if args.config == 4:
        from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, allocate_stats, make_telemetry
        lo, hi = (int(x) for x in args.events.split(","))
        tspec = TelemetrySpec(seed=args.seed + 7, min_events=lo, max_events=hi)
        tele = [make_telemetry(tspec, windows[w], K, base=(w * world + rank) * M) for w in range(n_windows)]
        stats = allocate_stats(M, K, dev)
        n_events = sum(t.num_events for t in tele) / n_windows
    if args.emulate_allreduce and (world > 1 or not args.force_merge or cpu):
        raise SystemExit("bench: --emulate-allreduce prices N ranks on ONE GPU (needs --force-merge, N = 1)")
    # the causal record correction where the uncorrected records miss the fidelity bar
    # (records median |d mu| <= 15 against exact sequential rating): 12.6 at N = 2, 27.3 at
    # N = 4, 29.6 at N = 8 uncorrected (k = N, profiles/r4/dp_accuracy_records.log), 7.85
    # corrected at N = 8 (profiles/r5/dp_gloo_rehearsals.log) -- so N >= 4, or the emulated
    # N of a one-GPU projection; ANA_DP_CORRECT_RECORDS overrides
    n_eff = world if world > 1 else (int(args.emulate_allreduce.split(":")[0]) if args.emulate_allreduce else 0)
    correct = None if os.environ.get("ANA_DP_CORRECT_RECORDS") is not None or not n_eff else n_eff >= 4
    merger = (SweepMerger(P, dev, comm_dtype=args.comm_dtype, sweeps=args.sweeps, force=args.force_merge,
                          emulate=args.emulate_allreduce, correct_records=correct)
              if world > 1 or args.force_merge else None)
    auto_mode = args.telemetry_mode == "auto"
    tele_path = None
    if tele is not None and auto_mode:
        tele_path = "fused (inline)"
    if tele is not None and auto_mode and not rater.fuses((tele[0].evoff, tele[0].events, stats), Mw):
        tele_path = "MFMA kernel after the rating (launch > ANA_TELE_FUSE_MAX)"
        # window-sized launches: the MFMA kernel on its own stream, started once the
        # rating has claimed 0.5 of its chunks (beside the rest of the rating, its drain
        # and the next prepass, which the same signal starts when it overlaps): 8.62 ms
        # against 8.79 from 0.7 and 8.85 with a serial prepass (profiles/r5/
        # prepass_overlap_grid256.log; round 4 at two waves per SIMD: 0.4 best, 9.54-9.56 vs
        # 9.67-9.70 from 0.8 and 9.85 behind the rating, config4_tail_point_and_c3_warm.log);
        # needs hipStreamWaitValue64
        from analyzer_amd.ops.native import native as _native

        if not cpu and _native().can_wait_value(dev.index or 0):
            args.telemetry_mode = "tail"
            tele_path = ("MFMA kernel on its own stream from %s of the rating's chunks (launch > "
                         "ANA_TELE_FUSE_MAX)" % (os.environ.get("ANA_TELE_TAIL_AT") or "0.2"))
    tail_at = float(os.environ.get("ANA_TELE_TAIL_AT") or (0.2 if auto_mode else 0.9)) \
        if tele is not None and args.telemetry_mode == "tail" else 0.0
    pipe = WindowPipeline(rater, roster, K, merger=merger, signal_at=tail_at,
                          telemetry=tele is not None and args.telemetry_mode == "fused")
    # the DP merge corrects window i's records during window i+1's collective
    # (parallel/sweep.py defer): records double-buffered, so window i+1's rating
    # writes the other buffer (a consumer streams the records out of the idle one)
    outs = [out, RateResult.allocate(Mw, K, dev)] if merger is not None and merger.correct and \
        merger.defer else [out]
    rater.clear_sticky(dev)  # executor error flags, OR-ed over every launch of the run
    sync()
    D = pipe.depth  # windows prepared ahead (runtime/engine.py)
    prepared = {j: pipe.prepare(windows[j % n_windows]) for j in range(min(D, total_windows))}

    tstream = None
    ttail = None
    if tele is not None and args.telemetry_mode == "tail":
        ttail = torch.cuda.Stream(dev)
        if not pipe._signal:
            raise SystemExit("--telemetry-mode tail needs hipStreamWaitValue64 on this device")
    if tele is not None and args.telemetry_mode == "overlap":
        # ANA_TELE_CUS=n: the co-running aggregation confined to n CUs (HIP CU mask),
        # so it takes bandwidth without slowing every executor wave
        n_cus = int(os.environ.get("ANA_TELE_CUS") or 0)
        if n_cus > 0:
            from analyzer_amd.ops.native import native

            tstream = torch.cuda.ExternalStream(native().cu_masked_stream(dev.index or 0, n_cus), device=dev)
        else:
            tstream = torch.cuda.Stream(dev)

    def step(i):
        out = outs[i % len(outs)]
        # rate window i, then the prepass of window i+D on the side stream behind
        # its tail (every timed step carries exactly one prepass and one rating)
        nxt = windows[(i + D) % n_windows]
        if ttail is not None:
            # the telemetry of window i beside the tail of its rating and the next
            # prepass; rating i + 1 waits for it (no co-run with a full executor)
            main = torch.cuda.current_stream(dev)
            if i > 0:
                main.wait_stream(ttail)
            produced = torch.cuda.Event()
            produced.record(main)
            res_prep = pipe.step(prepared.pop(i), nxt, out=out)
            ttail.wait_event(produced)
            pipe.wait_tail(ttail)
            with torch.cuda.stream(ttail):
                aggregate(tele[i % n_windows], K, stats)
            prepared[i + D] = res_prep[1]
            return
        if tstream is not None:
            # window i's telemetry co-runs with its rating; the step ends when both have
            main = torch.cuda.current_stream(dev)
            tstream.wait_stream(main)
            with torch.cuda.stream(tstream):
                aggregate(tele[i % n_windows], K, stats)
            _, prepared[i + D] = pipe.step(prepared.pop(i), nxt, out=out)
            main.wait_stream(tstream)
        elif tele is None or args.telemetry_mode == "separate":
            _, prepared[i + D] = pipe.step(prepared.pop(i), nxt, out=out)
            if tele is not None:
                aggregate(tele[i % n_windows], K, stats)
        else:
            t = tele[i % n_windows]
            _, prepared[i + D] = pipe.step(prepared.pop(i), nxt, out=out,
                                           telemetry=(t.evoff, t.events, stats))

    per = sub  # loop units (windows) per step
    for i in range(args.warmup * per):
        step(i)
    pipe.finish()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    if merger is not None:
        merger.timing = True  # stage events on the main stream (no syncs)
    t0 = time.perf_counter()
    for i in range(args.warmup * per, total_windows):
        step(i)
    pipe.finish()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    ms = elapsed * 1000.0 / args.steps
    merge = {}
    side_correct = None
    if merger is not None:
        merger.timing = False
        merge = {k: v / args.steps for k, v in merger.stage_ms().items()}
        if merger.split() and merger.correct and (world > 1 or args.force_merge):
            # the split merge corrects the records on a side stream beside the next rating:
            # its own time, off the main stream (parallel/sweep.py merge_split)
            side_correct = merger.correction_ms() / args.steps
    vals = [ms] + [merge.get(k, 0.0) for k in ("messages", "allreduce", "apply", "overlap", "correct")] + \
        [side_correct or 0.0]
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t[0].item())
    merge_ms = None
    if merger is not None:
        mm = [float(x) for x in t[1:].tolist()]
        # snapshot: 0 -- the merge decodes into the roster and the next window's
        # start in one pass, so no per-window copy of the roster is taken
        # prepass_overlap: the next window's prepass, enqueued while the all-reduces
        # are in flight (serial placement); "allreduce" is what stays exposed after it
        split = merger.split()
        merge_ms = {"snapshot": 0.0, "messages": mm[0], "allreduce": mm[1], "apply": mm[2],
                    # the causal record correction's pass over the window's records: on the main
                    # stream (round-5 merges), or beside the next rating (split merge: side-stream
                    # time, not part of "total")
                    "correct_records": (mm[5] if split else mm[4]) if merger.correct else None,
                    "correct_records_on": ("side stream beside the next rating" if split else "main stream")
                    if merger.correct else None,
                    "collective": ("split: all-to-all + owner reduce + all-gather of the sum (critical), "
                                   "prefix all-to-all deferred" if split else "scan (3 (N-1)/N)" if merger.correct
                                   else "bucketed all-reduce"),
                    "total": sum(mm[:3]) + (0.0 if split else mm[4]), "prepass_overlap": mm[3],
                    "bytes_per_rank": merger.comm_bytes,
                    "buckets": len(merger.buckets()),
                    # where the next window's prepass ran: beside the merge (serial) or in
                    # the rating's tail; chosen from a timed all-reduce for N > 1
                    "prepass_placement": "beside the merge" if pipe.serial else "rating tail %.2f" % pipe.tail,
                    "allreduce_probe_ms": pipe.allreduce_probe_ms}
    if merger is not None:
        merger.check()  # a clamped merge decode fails the run, as the executor's flags do
    flags = rater.sticky_flags(dev).cpu()
    if int(flags.sum()):
        raise RuntimeError("dataflow error flags set during the benchmark: %s" % flags.tolist())
    if args.check:
        out = outs[(total_windows - 1) % len(outs)]
        counts = out.status_counts()
        assert NOT_PROCESSED not in out.status.unique().tolist(), counts
        if rank == 0:
            print("status counts (last window):", counts, file=sys.stderr)
    verify = None
    if args.verify and rank == 0:  # untimed: a fresh roster and window 0, device vs fp64 host
        from analyzer_amd.ops.verify import verify_window

        verify = verify_window(make_roster(RosterSpec(num_players=P, seed=args.seed), device=dev),
                               windows[0], K)
        if tele is not None:
            verify["note"] = "rating only (telemetry is checked by tests/test_telemetry.py)"
    accuracy = None
    if world > 1 and args.accuracy and rank == 0 and args.config != 4:
        # untimed: the error this run's settings leave against the exact sequential
        # result -- the same N, roster, slice length, merges, sweeps and message dtype,
        # the N ranks simulated with the same kernels on this GPU (parallel/accuracy.py)
        from analyzer_amd.parallel.accuracy import run as accuracy_run

        t_acc = time.perf_counter()
        tab = accuracy_run(world, P, Mw, sub, [args.sweeps], device=dev, team_size=K, seed=args.seed,
                           comm_dtype=args.comm_dtype, p_rated=RosterSpec().p_rated, warm_windows=1)
        st = tab["sweeps"][str(args.sweeps)]
        sh = st["tracks"].get("shared", {})
        accuracy = {"vs": "exact sequential rating of the same %d x %d matches (one step)" % (world, M),
                    "shared_dmu_median": sh.get("dmu_median"), "shared_dmu_p99": sh.get("dmu_p99"),
                    "shared_dmu_max": sh.get("dmu_max"),
                    "spearman_mu_minus_sigma": sh.get("spearman_mu_minus_sigma"),
                    "sigma_ratio_p01_p99": [sh.get("sigma_ratio_p01"), sh.get("sigma_ratio_p99")],
                    "records_dmu_median": st.get("records_shared_mu", {}).get("dmu_median"),
                    "records_dmu_p99": st.get("records_shared_mu", {}).get("dmu_p99"),
                    "records_dmu_max": st.get("records_shared_mu", {}).get("dmu_max"),
                    "merge_clamp_hits": st.get("clamp_hits"),
                    "seconds": round(time.perf_counter() - t_acc, 2)}
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's untimed accuracy pass
    value = world * M / (ms / 1000.0)
    metric = "matches/sec rated (whole node), 3v3 TrueSkill, 1M-player roster"
    extra = {}
    if args.config == 3:
        metric = "matches/sec rated (whole node), 5v5 TrueSkill, 1M-player roster, DP sweep merge"
    if args.config == 5:
        metric = ("matches/sec re-rated (whole node), full-history windows, 3v3 TrueSkill, "
                  "10M-player roster")
    if args.config == 4:
        metric = ("matches/sec rated + telemetry aggregated (whole node), 3v3 TrueSkill, "
                  "1M-player roster, streaming")
        extra = {"events_per_match": n_events / M, "events_per_s": world * n_events / (ms / 1000.0),
                 "telemetry_mode": "auto" if auto_mode else args.telemetry_mode}
        if auto_mode:
            extra["telemetry_path"] = tele_path
    if rank == 0:
        print(json.dumps({
            "metric": metric,
            "value": value,
            "unit": "matches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / (BASELINE_5V5_MATCHES_PER_S if args.config == 3
                                    else BASELINE_MATCHES_PER_S),
            "dtype": "fp32",
            "data": "synthetic (on-device counter RNG stream, random-init %d-player roster)" % P,
            "merge_ms": merge_ms,
            # how the step was scheduled: the executor's grid (ops/rate.py launch_blocks) and
            # where the next window's prepass ran (runtime/engine.py placement)
            "schedule": {"executor_workgroups": pipe.grid,
                         "prepass": ("serial" if pipe.serial else "rating tail %.2f" % pipe.tail)},
            "verify": verify,
            "accuracy": accuracy,
            "rccl_world": dist.get_world_size() if world > 1 else None,
            "dist_backend": backend if world > 1 else None,
            "device": dev.type,
            "config": {
                "model": "TrueSkill 2-team EP (beta=1000, tau=10, draw_probability=0), "
                         "shared + per-mode tracks",
                "global_batch": world * M,
                "seq_len": 2 * K,
                "players": P,
                "matches_per_gpu": M,
                "merges_per_step": sub,
                "team_size": K,
                "parallelism": "dp%d" % world,
                "mode": ("exact" if world == 1 else
                         "sweep (exact per rank + %s posterior merge, %d causal sweep%s)"
                         % ("RCCL" if backend == "nccl" else backend, args.sweeps, "s" if args.sweeps > 1 else "")),
                "bench_config": args.config,
                "skew": args.skew,
                "comm_dtype": args.comm_dtype if world > 1 or args.force_merge else None,
                "force_merge": bool(args.force_merge),
                "emulated_allreduce": args.emulate_allreduce,
                "sweeps": args.sweeps if world > 1 else None,
                **extra,
            },
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
