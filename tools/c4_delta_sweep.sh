#!/bin/bash
# C4 global-label kernel: rows 0-4095 under bucket widths (ns), DELTAS="6000000 10000000 ..."
cd "$(dirname "$0")/.."
for d in ${DELTAS:-6000000 8000000 10000000 12500000 15000000}; do
  SHD_SSSP_DELTA=$d timeout -k 10 200 python -u tools/c4_probe.py 0 4096 3 || exit 3
done
