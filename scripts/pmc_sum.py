"""Sum rocprofv3 counter values of the executor dispatches (rate_dataflow_kernel)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc2"
agg = collections.OrderedDict()
for f in sorted(glob.glob(root + "/*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "rate_dataflow" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, v in agg.items():
    print("%-28s %16.0f" % (k, v))
