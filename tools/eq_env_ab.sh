#!/bin/bash
# A/B of a knob (environment variable, read at shd_open) on the C5 relay + event-queue leg:
#   tools/eq_env_ab.sh VAR v1 v2 ...   (each value twice, alternated)
cd "$(dirname "$0")/.."
var=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 150 python3 bench.py --steps 5 --no-cpu-baseline --no-c3 --no-c4 --no-codel \
      --no-tbucket --no-e2e 2>/dev/null > gpurun_out/eqab.json || exit 3
    python3 - "$var=$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/eqab.json").readline()); e = d["relay"]["equeue"]
print(sys.argv[1], "advance", round(e["advance_ms_per_round"], 4), "relay+merge", round(e["ms_per_round"], 4),
      "each", e["advance_ms_each"])
PY
  done
done
