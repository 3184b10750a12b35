#!/usr/bin/env python3
"""Time the standalone K8 telemetry aggregation (and its diagnostic / A-B
variants, ANA_TELE_DEBUG / ANA_TELE_IMPL) interleaved in one process, and check
each variant's output against the default kernel on the same events."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from analyzer_amd.ops.synth import StreamSpec, make_stream  # noqa: E402
from analyzer_amd.ops.telemetry import TelemetrySpec, aggregate, allocate_stats, make_telemetry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matches", type=int, default=10_000_000)
    ap.add_argument("--players", type=int, default=1_000_000)
    ap.add_argument("--team-size", type=int, default=3)
    ap.add_argument("--events", default="20,60")
    ap.add_argument("--variants", default="impl0,impl1,dbg1,dbg2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    # dbg<D> and non-default spans live in the diagnostic library only
    # (python -m analyzer_amd.build_ext --diag -> analyzer_amd/_C_diag*.so)
    diag = any(v.startswith("dbg") or (v.partition("s")[2] not in ("", "63")) for v in args.variants.split(","))
    if diag and not os.environ.get("ANA_NATIVE_LIB"):
        import glob

        libs = glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "analyzer_amd", "_C_diag*.so"))
        if not libs:
            sys.exit("variants %s need the diagnostic library: python -m analyzer_amd.build_ext --diag"
                     % args.variants)
        os.environ["ANA_NATIVE_LIB"] = libs[0]
    dev = torch.device("cuda:0")
    M, K = args.matches, args.team_size
    rec = make_stream(StreamSpec(team_size=K, seed=5), M, args.players, device=dev)
    lo, hi = (int(x) for x in args.events.split(","))
    tel = make_telemetry(TelemetrySpec(seed=9, min_events=lo, max_events=hi), rec, K)
    E = tel.num_events
    ref = aggregate(tel, K)
    torch.cuda.synchronize()
    stats = allocate_stats(M, K, dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    res = {}
    for rnd in range(args.rounds):
        for v in args.variants.split(","):
            # variant: impl<I> or dbg<D>, optionally s<SPAN> (e.g. impl1s32, dbg7s63)
            name, _, span = v.partition("s")
            os.environ["ANA_TELE_DEBUG"] = name[3:] if name.startswith("dbg") else "0"
            os.environ["ANA_TELE_IMPL"] = name[4:] if name.startswith("impl") else "1"
            if span:
                os.environ["ANA_TELE_SPAN"] = span
            else:
                os.environ.pop("ANA_TELE_SPAN", None)
            stats.zero_()
            bad.zero_()
            aggregate(tel, K, stats, bad)
            torch.cuda.synchronize()
            err = float((stats - ref).abs().max() / ref.abs().max().clamp_min(1))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(args.iters):
                aggregate(tel, K, stats, bad)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / args.iters
            gbs = (E * 16 + M * 2 * K * 8 * 4 + (M + 1) * 8) / ms / 1e6
            r = res.setdefault(v, {"ms": [], "rel_err": err, "bad": int(bad.item())})
            r["ms"].append(ms)
            print("round %d %-6s %7.3f ms  %6.0f GB/s  rel err vs default %.2e  bad %d"
                  % (rnd, v, ms, gbs, err, int(bad.item())), flush=True)
    print(json.dumps({"matches": M, "events": E, "K": K,
                      "by_variant": {k: {"ms_min": min(v["ms"]), "rel_err": v["rel_err"]}
                                     for k, v in res.items()}}))


if __name__ == "__main__":
    main()
