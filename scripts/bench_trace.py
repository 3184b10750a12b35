"""Timeline of the last bench steps from a rocprofv3 kernel trace (queue = stream)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tprof/run_kernel_trace.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print("%9.3f %9.3f %7.3f q%s %s" % (s, e, e - s, r.get("Queue_Id", ""), r["Kernel_Name"][:70]))
