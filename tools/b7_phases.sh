#!/bin/bash
# Pipeline-7 K4 phase timing: bin_sort_v7 stopped after each phase (SHD_B7_STOP = 1 load,
# 2 look-back, 3 grouping, 4 sorts; 0 = full), kernel stats per run, then the relay parity
# tests.  The stopped runs' outputs are wrong by design; only their kernel times are read.
set -e
for st in ${B7_STOPS:-0 3 4}; do
  SHD_B7_STOP=$st timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st$st -o run -- python tools/relay_only.py 10 > gpurun_out/st$st.log 2>&1
done
timeout -k 10 200 python -u -m pytest tests/test_relay_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rt.log 2>&1
