#!/bin/bash
# A/B of a knob on C4 rows [rb, re) (tools/c4_probe.py, delta-stepping), alternated twice:
#   tools/c4_env_ab.sh VAR rb re v1 v2 ...
cd "$(dirname "$0")/.."
var=$1; rb=$2; re=$3; shift 3
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 200 python3 tools/c4_probe.py $rb $re 3 2>/dev/null | sed "s/^/$var=$v /" | cut -c1-140 || exit 3
  done
done
