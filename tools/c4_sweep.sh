#!/bin/bash
# C4 global-label kernel sweep (one GPU): flat expansion on/off, slots per CU, bucket bytes
set -e
cd "$(dirname "$0")/.."
for slots in 1 2 4; do
  SHD_SSSP_SLOTS=$slots timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3,1
done
SHD_SSSP_FLAT=0 SHD_SSSP_SLOTS=2 timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3
SHD_SSSP_NO_BKT=1 SHD_SSSP_SLOTS=2 timeout -k 10 120 python -u tools/c4_probe.py 0 4096 3
