"""Kernel averages (us) per sweep value: python tools/sweep_summary.py v1 v2 ... (gpurun_out/sw_<v>)."""
import csv
import sys

for v in sys.argv[1:]:
    row = []
    for r in csv.DictReader(open(f"gpurun_out/sw_{v}/run_kernel_stats.csv")):
        n = r["Name"].split("(")[0].replace("void ", "").replace("shd::", "")
        if any(k in n for k in ("stamp", "bin_", "relay_", "draws")):
            row.append(f"{n[:16]}={float(r['AverageNs']) / 1e3:.1f}")
    ms = [l for l in open(f"gpurun_out/sw_{v}.log") if l.startswith("ms_per_round")]
    print(v, ms[-1].strip() if ms else "?", " ".join(row))
