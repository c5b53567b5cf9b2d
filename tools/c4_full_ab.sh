#!/bin/bash
# full C4 build (bench c4 leg) alternating bucket widths (ns) on one box: DELTAS="a b a b"
cd "$(dirname "$0")/.."
for d in ${DELTAS:-6018057 10030095 6018057 10030095}; do
  SHD_SSSP_DELTA=$d timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-relay --no-c3 --no-codel --no-tbucket --no-e2e --no-c5b 2>/dev/null > gpurun_out/c4full.json || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/c4full.json').read().strip().splitlines()[-1]); print('delta $d', round(d['c4']['ms_per_build'],1))"
done
