#!/bin/bash
# A/B of tuning builds (SHD_ACCEL_LIB) on C3 (10k-node BA, DELTA) and the C2 step, alternated twice:
#   tools/c3_lib_ab.sh <lib.so|default> ...
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset SHD_ACCEL_LIB; else export SHD_ACCEL_LIB=$lib; fi
    c3=$(PROBE_GRAPH=c3 timeout -k 10 120 python3 tools/c2_probe.py 3 2>/dev/null | grep same=) || exit 3
    c2=$(timeout -k 10 120 python3 tools/c2_probe.py 0 2>/dev/null | grep same=) || exit 3
    echo "$(basename $lib) C3: $c3 | C2: $c2"
  done
done
