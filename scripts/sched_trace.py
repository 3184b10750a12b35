"""Print the last schedule prepass of a rocprofv3 kernel trace (gpurun_out/sprof)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sprof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "fillBuffer" in r["Kernel_Name"]]
last = rows[starts[-2]:] if len(starts) >= 2 else rows
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print("%8.1f %8.1f us %7.1f %s" % (s, e, e - s, r["Kernel_Name"][:80]))
print("total %.1f us" % ((int(last[-1]["End_Timestamp"]) - t0) / 1e3))
