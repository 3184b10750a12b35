#!/usr/bin/env python3
"""Per-kernel time summary of a rocprofv3 results database (rocpd sqlite).

    python scripts/rocpd_summary.py gpurun_out/prof/run_results.db [--last N] [--match substr]

Prints each dispatch of the last N (default all) in order with its duration,
then the per-kernel totals (calls, total / mean ms)."""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name.replace("ana::", "").replace("(anonymous namespace)::", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select k.kernel_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from "
                     "rocpd_kernel_dispatch d join rocpd_info_kernel_symbol k on d.kernel_id = k.id "
                     "order by d.start").fetchall()
    rows = [r for r in rows if a.match in r[0]]
    if a.last:
        rows = rows[-a.last:]
        t0 = rows[0][1]
        for name, s, e, g, w in rows:
            print("%10.3f %8.3f ms  grid %8d  %s" % ((s - t0) / 1e6, (e - s) / 1e6, g // max(w, 1), short(name)))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, _, _ in rows:
        tot[short(name)][0] += 1
        tot[short(name)][1] += (e - s) / 1e6
    print("%-90s %6s %10s %9s" % ("kernel", "calls", "total ms", "mean ms"))
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print("%-90s %6d %10.3f %9.4f" % (k, n, t, t / n))


if __name__ == "__main__":
    main()
