#!/bin/bash
# A/B of a relay knob (environment variable, read at shd_open) on the C5 relay leg, alternated twice:
#   tools/relay_env_ab.sh VAR v1 v2 ...
cd "$(dirname "$0")/.."
var=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 150 python3 bench.py --steps 10 --no-cpu-baseline --no-c3 --no-c4 --no-codel \
      --no-tbucket --no-e2e --no-equeue 2>/dev/null > gpurun_out/reab.json || exit 3
    python3 - "$var=$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/reab.json").readline()); r = d["relay"]
print(sys.argv[1], "relay ms/round", round(r["ms_per_round"], 4))
PY
  done
done
