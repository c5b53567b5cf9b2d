#!/bin/bash
# WRITE_SIZE of the relay kernels per round (10 C5 rounds, tools/relay_only.py) under a knob:
#   tools/relay_write_ab.sh VAR v1 v2 ...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/rwab_$v -o run -- \
    python3 tools/relay_only.py 10 > gpurun_out/rwab_$v.log 2>&1 || exit 3
  python3 - gpurun_out/rwab_$v "$var=$v" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1] + "/run_counter_collection.csv")):
    acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k in ("void shd::relay_stamp_v6<true>", "shd::bin_sort_v7", "shd::relay_draws"):
    v = acc.get(k, [])
    if v:
        print(sys.argv[2], k, "MB/launch", round(sum(v) / len(v) / 1e3, 1))
PY
done
