"""Per-kernel totals and the per-window timeline of a rocprofv3 kernel trace:
python scripts/prof_summary.py run_kernel_trace.csv [last N rows of the timeline]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 40
agg = collections.OrderedDict()
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    c, t = agg.get(n, (0, 0.0))
    agg[n] = (c + 1, t + d)
print("%-72s %6s %10s %9s" % ("kernel", "calls", "total ms", "avg ms"))
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-72s %6d %10.3f %9.3f" % (n, c, t, t / c))
t0 = int(rows[0]["Start_Timestamp"])
print("\ntimeline (ms since the first dispatch), last %d dispatches" % tail)
for r in rows[-tail:]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    print("%-48s q%-3s %10.3f %10.3f %8.3f" % (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-48:], r.get("Queue_Id", ""), s, e, e - s))
