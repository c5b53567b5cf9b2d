#!/bin/bash
# bin_sort_v7<false> (plain round) against bin_sort_v7<true> (sharded, world 1 only) per phase:
# the sharded probe under a kernel trace with SHD_B7_STOP = 0 (whole kernel) .. 4 (tuning only:
# the kernel stops after that phase, wrong output); medians of the timed rounds.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in 0 1 2 3 4; do
  SHD_B7_STOP=$st timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_b7x_$st -o run \
    -- python3 tools/sharded_round_probe.py 4 > gpurun_out/r06_b7x_$st.log 2>&1 || { tail -5 gpurun_out/r06_b7x_$st.log; exit 3; }
  python3 - $st <<'PY'
import csv, statistics, sys
st = sys.argv[1]
t = {"false": [], "true": []}
for r in csv.DictReader(open(f"gpurun_out/r06_b7x_{st}/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    for k in t:
        if f"bin_sort_v7<{k}>" in n:
            t[k].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
f = [d for _, d in sorted(t["false"])][2:]          # the plain leg's timed rounds
w1 = [d for _, d in sorted(t["true"])][2:6]         # the world-1 leg's timed rounds (4 + 2 warm-up)
print(f"stop={st}: bin_sort_v7<false> {statistics.median(f):.1f} us, bin_sort_v7<true> (world 1) {statistics.median(w1):.1f} us")
PY
done
