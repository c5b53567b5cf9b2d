#!/bin/bash
# C4 global-label kernel: rows 0-4095 under slot counts per CU and lane-group widths (tuning)
cd "$(dirname "$0")/.."
for s in ${SLOTS:-1 2 3}; do
  for g in ${GS:-4 8}; do
    SHD_SSSP_SLOTS=$s SHD_SSSP_G=$g timeout -k 10 200 python -u tools/c4_probe.py 0 4096 3 || exit 3
  done
done
