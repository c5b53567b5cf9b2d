#!/bin/bash
# C3 (10k-node BA) full DELTA builds under bucket widths (ns): DELTAS="a b c"
cd "$(dirname "$0")/.."
for d in ${DELTAS:-6000000 12500000 25000000 40000000}; do
  SHD_SSSP_DELTA=$d timeout -k 10 200 python -u tools/c3_probe.py || exit 3
done
timeout -k 10 200 python -u tools/c3_probe.py
