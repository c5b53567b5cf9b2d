"""Print the relay kernels of rocprofv3 --stats CSVs: python tools/kstats.py dir [dir ...]"""
import csv
import sys

for d in sys.argv[1:]:
    print("==", d)
    for x in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        n = x["Name"]
        if any(k in n for k in ("stamp", "bin_sort", "hist", "col_scan", "base_scan", "draws", "eqr_")):
            print("  %-48s %5s %9.1f us" % (n[:48], x["Calls"], float(x["AverageNs"]) / 1e3))
