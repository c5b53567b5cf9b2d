#!/bin/bash
# Generic A/B of an environment toggle over a probe script:
#   AB_VAR=NAME tools/env_ab.sh "<probe command>" v1 v2 ...   (each value twice, alternating)
cd "$(dirname "$0")/.."
var=${AB_VAR:?AB_VAR}
cmd=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 300 $cmd 2>/dev/null | awk -v p="$var=$(basename "$v")" '{print p, $0}' || exit 3
  done
done
