#!/bin/bash
# A/B of tuning builds (SHD_ACCEL_LIB) on the C5 relay and relay + queue legs, alternated twice:
#   tools/relay_lib_ab.sh <lib.so|default> ...
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset SHD_ACCEL_LIB; else export SHD_ACCEL_LIB=$lib; fi
    timeout -k 10 150 python3 bench.py --steps 5 --no-cpu-baseline --no-c3 --no-c4 --no-codel --no-tbucket \
      --no-e2e 2>/dev/null > gpurun_out/rlab.json || exit 3
    python3 - "$(basename $lib)" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/rlab.json").readline()); r = d["relay"]; e = r["equeue"]
print(sys.argv[1], "relay ms/round", round(r["ms_per_round"], 4), "advance", round(e["advance_ms_per_round"], 4),
      "relay+merge", round(e["ms_per_round"], 4), "C2", round(d["ms_per_step"], 4))
PY
  done
done
