"""Sum rocprofv3 counter values per counter over the dispatches of kernels whose
name contains a substring: python scripts/pmc_kernel.py <dir-glob> <substring>."""
import collections
import csv
import glob
import sys

root, sub = sys.argv[1], sys.argv[2]
agg = collections.OrderedDict()
for f in sorted(glob.glob(root + "/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, v in agg.items():
    print("%-28s %18.0f" % (k, v))
