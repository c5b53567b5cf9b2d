#!/bin/bash
# A/B of tuning builds (SHD_ACCEL_LIB) on the C2 build and C4 rows 0-4095, alternated twice:
#   tools/lib_ab.sh <lib.so|default> ...
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset SHD_ACCEL_LIB; else export SHD_ACCEL_LIB=$lib; fi
    timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-relay \
      --no-c3 --no-c4 --no-codel --no-tbucket --no-e2e 2>/dev/null > gpurun_out/libab.json || exit 3
    c2=$(python3 -c "import json; d=json.loads(open('gpurun_out/libab.json').readline()); print(round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4))")
    c4=$(timeout -k 10 120 python3 tools/c4_probe.py 0 4096 3 2>/dev/null | sed 's/.*ms_main=\([0-9.]*\).*same=\([A-Za-z]*\).*/\1 \2/') || exit 3
    echo "$(basename $lib) C2 step/kernel $c2  C4 rows0-4095 $c4"
  done
done
