"""Reduce rocprofv3 --pmc passes to one CSV: mean counter value per dispatch of the kernels whose
name contains a filter string.   python tools/pmc_summary.py <out.csv> <filter> <dir> [<dir> ...]"""
import csv
import sys
from collections import defaultdict

out, filt, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
acc = defaultdict(list)
for d in dirs:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if filt in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "counter", "dispatches", "mean_per_dispatch"])
    for (k, c), v in sorted(acc.items()):
        w.writerow([k, c, len(v), round(sum(v) / len(v), 1)])
print(open(out).read())
