#!/bin/bash
# C4 row-range A/B of an environment toggle: AB_VAR=NAME [ROWS="0 4096"] tools/c4_ab.sh v1 v2 ...
# (each value twice, alternating; the printed hash must agree across values)
cd "$(dirname "$0")/.."
var=${AB_VAR:?AB_VAR}
rows=${ROWS:-0 4096}
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 300 python3 tools/c4_probe.py $rows 3 2>/dev/null | awk -v p="$var=$(basename $v)" '{print p, $0}' || exit 3
  done
done
